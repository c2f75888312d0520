/*
 * cbf_amd.h -- C ABI of the MI355X-native CBF safety filter (libcbf_amd.so).
 *
 * Drop-in boundary for the reference's hot path (YilunAllenChen/CBF):
 *   ControlBarrierFunction.__init__        cbf.py:6-16            -> cbf_params_init
 *   ControlBarrierFunction.get_safe_control cbf.py:18-92          -> cbf_get_safe_control_batch
 *   (A, b) handed to cvxopt.solvers.qp     cbf.py:64-81           -> cbf_assemble_rows
 *   per-agent cull + filter loop           cross_and_rescue.py:135-160,
 *                                          meet_at_center.py:118-143 -> cbf_filter_allpairs / cbf_filter_cells
 *   Laplacian consensus / cyclic pursuit   cross_and_rescue.py:108-125,
 *                                          meet_at_center.py:86-103 -> cbf_consensus_csr / cbf_consensus_lattice
 *   Euler integration                      cross_and_rescue.py:173 -> cbf_euler
 *   whole timestep (large swarm)           cross_and_rescue.py:97-175 -> cbf_lattice_step
 *   batched Monte-Carlo rendezvous         meet_at_center.py:76-153 (x n_scen) -> cbf_mc_rollout
 *   cull alone (neighbour index sets)      cross_and_rescue.py:141-150 -> cbf_cull_allpairs
 *   Euclidean HOCBF barrier mode           (north star; replaces the rows of cbf.py:38-59)
 *                                             -> cbf_get_safe_control_batch_hocbf / cbf_filter_indexed_hocbf
 *
 * Conventions
 *  - All arrays are caller-owned DEVICE pointers (hipMalloc / torch CUDA tensors), fp64,
 *    row-major, contiguous: positions / velocities / controls are [n][2] (x, y), states [n][4]
 *    = (x, y, vx, vy) as in the reference's packed rows (cross_and_rescue.py:132-133).
 *  - Parameter structs (cbf_params, cbf_grid, cbf_diag) live in HOST memory.
 *  - `stream` is a hipStream_t (NULL = default stream).  Every call is asynchronous and
 *    stream-ordered; no call allocates, synchronises or keeps global state, so any sequence
 *    may be captured into a hipGraph.  Calls are re-entrant.
 *  - Return value: 0 on success, CBF_EINVAL (<0) on a bad argument (nothing launched),
 *    or a positive hipError_t from the launch.  No exception crosses the ABI.
 *  - Results are deterministic (no float atomics on any result path) and bit-identical to
 *    the CPU oracle in oracle/ for the same inputs.
 */
#ifndef CBF_AMD_H
#define CBF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBF_ABI_VERSION 7

#define CBF_EINVAL (-1)

/* per-ego status (low byte); bits 8..30 hold the number of +1 relaxations applied */
#define CBF_STATUS_IDLE 0           /* no neighbour: filter not run, u = u0 unclipped (cross_and_rescue.py:153) */
#define CBF_STATUS_OPTIMAL 1        /* exact minimiser of the QP of cbf.py:62-81 */
#define CBF_STATUS_RELAXED 2        /* infeasible; CBF rows relaxed by the cbf.py:84-87 rule, then optimal */
#define CBF_STATUS_BOX_INFEASIBLE 3 /* the 8 box rows alone are infeasible; x = 0 */
#define CBF_STATUS_RELAX_CAP 4      /* relaxation cap reached; x = 0 */
#define CBF_STATUS_NBR_OVERFLOW 5   /* indexed HOCBF filter: more neighbours than kmax; u = u0, not filtered */
#define CBF_STATUS_WORKSPACE_ERROR 6 /* the cell list of this step is unusable (its scan gave up waiting,
                                        which no correct launch should hit); u = u0, not filtered */

/* Rollout statistics of the lattice step (`stats`, device uint64[1024] zero-filled by the caller:
 * 64 slots of 16 words, slot i at stats + 16 i; sum the counts and take the maximum of the other
 * words over the slots).  Counted over the egos of the counted rows.  `stats` may be NULL in every
 * lattice entry point: nothing is recorded and the filter runs the instantiation that computes no
 * statistics (results are bit-identical either way; the reference computes none of them). */
#define CBF_STAT_SOLVES 0        /* agent-QP solves (egos with >= 1 neighbour) */
#define CBF_STAT_OPTIMAL 1       /* ... with status OPTIMAL (the reference's QP is feasible) */
#define CBF_STAT_RELAXED 2       /* ... RELAXED (infeasible as posed; the cbf.py:84-87 rule applied) */
#define CBF_STAT_INFEASIBLE 3    /* ... BOX_INFEASIBLE or RELAX_CAP */
#define CBF_STAT_SEIDEL 4        /* QPs queued for the full Seidel solve (neither the origin nor one projection) */
#define CBF_STAT_VIOL_OPTIMAL 5  /* max row violation over OPTIMAL QPs (bits of a double >= 0) */
#define CBF_STAT_VIOL_ORIGINAL 6 /* max violation of the ORIGINAL barrier rows over RELAXED QPs (bits) */
#define CBF_STAT_MIN_DIST2 7     /* 0x7FF0000000000000 - bits(min neighbour distance^2); 0 = no pair */
#define CBF_STAT_ERRORS 8        /* steps whose cell list was unusable (CBF_STATUS_WORKSPACE_ERROR) */
#define CBF_STAT_BINDING 9       /* QPs whose minimiser is not the origin (a barrier or box row binds) */
#define CBF_STAT_WIN_WALKS 10    /* window cull: egos whose neighbours were not lattice-near, found by the
                                    unbounded row walk (exact, slower; ABI 7) */
#define CBF_STAT_GUARD_STALLS 11 /* window cull: row-guard words read at their spin limit, i.e. as the
                                    worst bound (exact, slower; ABI 7) */

/* ControlBarrierFunction state (cbf.py:6-16) + the callers' dynamics and cull radius. */
typedef struct cbf_params {
    double max_speed; /* cbf.py:15 */
    double dmin;      /* cbf.py:12 (default 0.2) */
    double k;         /* cbf.py:13 (default 1) */
    double gamma;     /* cbf.py:16 (0.5, not a constructor argument in the reference) */
    double f[16];     /* dynamics f, row-major 4x4 (cross_and_rescue.py:31) */
    double g[8];      /* dynamics g, row-major 4x2 (cross_and_rescue.py:32) */
    double cull_t;    /* keep j iff |p_j - p_i|^2 < cull_t  <=>  sqrt(.) < safety_distance (:134,143) */
    double nrm[4][2]; /* derived: L_g = -hs_p @ g per sign quadrant q = (dx<0) | (dy<0)<<1 (cbf.py:56) */
    int32_t f_is_zero;/* derived */
    int32_t relax_cap;/* max +1 relaxations before CBF_STATUS_RELAX_CAP (default 65536) */
    /* Lattice steps (cbf_lattice_*): where the QPs that neither the origin nor one projection settles
     * are solved.  A window of at most solve_inline_max agents solves them inside the filter kernel;
     * a larger one queues them for a second kernel (one lane per QP).  Results are bit-identical
     * either way; only the speed differs.  < 0 (cbf_params_init's default): the library's own
     * threshold, 131072 agents (2 waves per SIMD on 256 CUs); 0: always queue.  ABI 4. */
    int32_t solve_inline_max;
    /* Bit CBF_LAUNCH_SEPARATE_GUARD: the window cull (CBF_RUN_WINDOW_CULL, cbf_lattice_window_*)
     * forms its row guard in a separate one-block kernel after the build instead of inside the
     * filter launch, whose blocks poll for it.  The in-launch form is the faster one on a GPU one
     * process owns; ranks that time-share one GPU should set the bit (a poll can wait for long
     * there).  Results are identical either way.  0 from cbf_params_init.  ABI 6 (was reserved). */
    uint32_t launch_flags;
} cbf_params;
#define CBF_LAUNCH_SEPARATE_GUARD 1u

/* Fill *p (host).  f16 / g8 may be NULL for the callers' f = 0, g = 0.1 [I2; 0]. */
int cbf_params_init(cbf_params* p, double max_speed, double dmin, double k, const double* f16, const double* g8,
                    double safety_distance);

/* Optional per-ego diagnostics (device pointers; any may be NULL).  Neighbour lists are
 * truncated at kmax entries (the count in nbr_count is never truncated). */
typedef struct cbf_diag {
    int32_t kmax;
    int32_t* nbr_idx;    /* [n_ego][kmax] entity indices, -1 padded */
    uint8_t* nbr_active; /* [n_ego][kmax] 1 if that neighbour's row is active at x */
    uint8_t* box_active; /* [n_ego] bit i = box row i (cbf.py:66 order) active */
    double* x;           /* [n_ego][2] QP deviation x (u = clip(x + u0)) */
    double* viol;        /* [n_ego] max_i (a_i.x - b_i), clipped at 0, over the final QP's rows */
} cbf_diag;

/*
 * get_safe_control (cbf.py:18-92) for a batch of independent egos with explicit
 * neighbour lists (CSR): ego i's neighbours are obs_states[nbr_off[i] .. nbr_off[i+1]).
 * robot_state [n][4], u0 [n][2], obs_states [M][4], u [n][2], status [n], x_out [n][2] (nullable).
 * An ego with zero neighbours still solves the 8-row box QP and is clipped.
 */
int cbf_get_safe_control_batch(const cbf_params* p, int32_t n_ego, const double* robot_state, const double* u0,
                               const int32_t* nbr_off, const double* obs_states, double* u, int32_t* status,
                               double* x_out, void* stream);

/* The (A, b) of cbf.py:72-80 per ego: rows [nbr_off[i] + 8 i, nbr_off[i+1] + 8 (i+1)) of
 * A [M + 8n][2] and b [M + 8n]: the ego's barrier rows in list order, then the 8 box rows. */
int cbf_assemble_rows(const cbf_params* p, int32_t n_ego, const double* robot_state, const double* u0,
                      const int32_t* nbr_off, const double* obs_states, double* A, double* b, void* stream);

/*
 * The per-agent loop of cross_and_rescue.py:135-160 over a swarm of n entities:
 * entities [0, n_obs) are obstacles, [n_obs, n) agents.  Egos are [ego_begin, ego_end)
 * (agents).  Ego e's state is (pos[e], vel[e]) and its nominal control is vel[e] (:133,155).
 * Neighbours: every obstacle with |dp|^2 < cull_t, every agent with 0 < |dp|^2 < cull_t.
 * Outputs are indexed e - ego_begin: u [n_ego][2] (= vel[e] unclipped if no neighbour),
 * status [n_ego], nbr_count [n_ego] (nullable).
 * _allpairs tests every entity (LDS-tiled); _cells uses a uniform cell list (grid below).
 */
int cbf_filter_allpairs(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos, const double* vel,
                        int32_t ego_begin, int32_t ego_end, double* u, int32_t* status, int32_t* nbr_count,
                        const cbf_diag* diag, void* stream);

/* cbf_filter_allpairs without diagnostics, for few egos against many entities: the candidate
 * range is split into chunks run by separate workgroups (so small n_ego still fills the GPU) and
 * the chunks' partial QP state is merged in order -- results identical to cbf_filter_allpairs.
 * Workspace: device memory of cbf_allpairs_workspace_size(n, n_ego) bytes, no initialisation. */
size_t cbf_allpairs_workspace_size(int32_t n, int32_t n_ego);
int cbf_filter_allpairs_split(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos, const double* vel,
                              int32_t ego_begin, int32_t ego_end, double* u, int32_t* status, int32_t* nbr_count,
                              void* workspace, size_t workspace_bytes, void* stream);

/* The cull of cross_and_rescue.py:141-150 alone: per ego e in [ego_begin, ego_end) its neighbour
 * indices in reference order (obstacles, then agents, ascending), the first kmax in
 * nbr_idx [n_ego][kmax] (-1 padded), the full count in nbr_count [n_ego]. */
int cbf_cull_allpairs(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos, int32_t ego_begin,
                      int32_t ego_end, int32_t kmax, int32_t* nbr_idx, int32_t* nbr_count, void* stream);

/*
 * Euclidean HOCBF barrier mode (no counterpart in the reference, which uses the sign-switched
 * L1 barrier of cbf.py:38-59).  Double integrator p' = v, v' = u; neighbours at constant
 * velocity; h = |p_i - p_j|^2 - dmin^2, psi1 = h' + a1 h, psi2 = psi1' + a2 psi1 >= 0 gives the
 * row (-2 dp) . u <= 2|dv|^2 + (a1 + a2) h' + a1 a2 h.  Box rows, +1 relaxation, de-bias and
 * clip are the reference's.  Each barrier row is its own half-plane (neighbour order).
 * Workspace: 32 bytes per barrier row (cbf_hocbf_workspace_size), rows are relaxed in place.
 */
typedef struct cbf_hocbf {
    double alpha1, alpha2; /* linear class-K gains of psi1 and psi2 */
} cbf_hocbf;

size_t cbf_hocbf_workspace_size(int64_t rows);

/* get_safe_control with HOCBF rows for a batch with explicit neighbour lists (CSR, as
 * cbf_get_safe_control_batch); the workspace must hold nbr_off[n_ego] rows. */
int cbf_get_safe_control_batch_hocbf(const cbf_params* p, const cbf_hocbf* hp, int32_t n_ego,
                                     const double* robot_state, const double* u0, const int32_t* nbr_off,
                                     const double* obs_states, double* u, int32_t* status, double* x_out,
                                     void* workspace, size_t workspace_bytes, void* stream);

/* The swarm loop with HOCBF rows over the neighbour lists of cbf_cull_allpairs: ego e's state is
 * (pos[e], vel[e]), u0 = vel[e]; no neighbour -> CBF_STATUS_IDLE, u = u0 unclipped; more than
 * kmax -> CBF_STATUS_NBR_OVERFLOW (rerun with a larger kmax).  Workspace: (ego_end - ego_begin)
 * * kmax rows.  x_out nullable. */
int cbf_filter_indexed_hocbf(const cbf_params* p, const cbf_hocbf* hp, int32_t n, const double* pos,
                             const double* vel, int32_t ego_begin, int32_t ego_end, int32_t kmax,
                             const int32_t* nbr_idx, const int32_t* nbr_count, double* u, int32_t* status,
                             double* x_out, void* workspace, size_t workspace_bytes, void* stream);

/* Uniform cell grid: cell (cx, cy) = clamp(floor((p - origin) * inv_h), 0, n-1).  The cell
 * edge 1/inv_h must be >= the cull radius (checked).  Clamping keeps results exact for
 * entities outside the grid (only speed suffers). */
typedef struct cbf_grid {
    double x0, y0;  /* origin */
    double inv_h;   /* 1 / cell edge */
    int32_t nx, ny; /* cells per axis */
} cbf_grid;

/* Workspaces (cells and lattice) must be zero-filled before their first use.  The first call binds
 * a workspace to its shape (the number of binned entities -- n, or W x win_rows -- and the grid's
 * cell count); it may then be reused by any sequence of calls of that shape on one stream (the
 * kernels restore what they consume: cell counts, queue counts, scan epochs).  A call with another
 * shape is detected on the device: every ego of it reports CBF_STATUS_WORKSPACE_ERROR (and the
 * lattice step counts it in CBF_STAT_ERRORS) until the workspace is zero-filled again. */
size_t cbf_cells_workspace_size(int32_t n, const cbf_grid* grid);

int cbf_filter_cells(const cbf_params* p, const cbf_grid* grid, int32_t n, int32_t n_obs, const double* pos,
                     const double* vel, int32_t ego_begin, int32_t ego_end, double* u, int32_t* status,
                     int32_t* nbr_count, const cbf_diag* diag, void* workspace, size_t workspace_bytes,
                     void* stream);

/*
 * Graph-Laplacian nominal control (cross_and_rescue.py:108-125, meet_at_center.py:86-103):
 *   out[k] = ( (sum_{t in row k} (src[col[t]] - src[self_offset + k])) [@ R] ) * scale
 * sum sequential from +0.0 in CSR order; R = [[rc, rs], [-rs, rc]] applied as the reference's
 * row-vector product when rotate != 0.  col[t] >= n_group addresses anchors[col[t] - n_group]
 * (the goal column of cross_and_rescue.py:102).  src [n_group][2], out [n_dst][2].
 */
int cbf_consensus_csr(int32_t n_dst, int32_t self_offset, int32_t n_group, const double* src, const double* anchors,
                      const int32_t* row_ptr, const int32_t* col, int32_t rotate, double rc, double rs,
                      double scale, double* out, void* stream);

/* 4-neighbour lattice Laplacian of a W x H lattice (ascending-index neighbour order),
 * rows [row_begin, row_end); pos holds lattice rows [pos_row0, ...) so that agent (r, c) is
 * pos[(r - pos_row0) W + c] (rows row_begin-1 .. row_end must be present where they exist);
 * out[(r - row_begin) W + c] = scale * sum. */
int cbf_consensus_lattice(int32_t W, int32_t H, int32_t row_begin, int32_t row_end, int32_t pos_row0,
                          const double* pos, double scale, double* out, void* stream);

/* pos <- pos + T * vel over n entities (cross_and_rescue.py:173). */
int cbf_euler(int32_t n, double* pos, const double* vel, double T, void* stream);

/*
 * One full timestep of a lattice swarm (SURVEY cfg3/cfg4): nominal control by the lattice
 * Laplacian (scale gain), cell-list cull, barrier assembly, exact QP, clip and Euler, for the
 * agents of rows [row_begin, row_end) of a W x H lattice (cross_and_rescue.py:97-175 shape).
 * pos holds rows [win_row0, win_row0 + win_rows) (a halo window when sharded; the window must
 * contain the owned rows plus one lattice row on each side where it exists).  Only owned rows
 * are written (index (r - row_begin) W + c): pos_out = p + T u (may alias or overlap pos: the
 * advance phase reads only cell-sorted copies), vel_out = nominal control, u = filtered control, status,
 * nbr_count (nullable).  Window agents whose nominal control cannot be formed (first / last
 * window row unless it is a lattice edge) are not candidates; callers size the halo so that
 * they are out of cull range and check it with `extents` (nullable, device double[4]):
 * {min y, max y} of the new owned positions, {max y over owned rows < row_end - guard_rows,
 * min y over owned rows >= row_begin + guard_rows}.  solves (nullable, device uint64[1024])
 * accumulates the number of agent-QP solves (egos with >= 1 neighbour) in slots [16 i], i < 64.
 *
 * cbf_lattice_step = cbf_lattice_build (nominal control + cell list) then cbf_lattice_advance
 * (filter + clip + Euler, the dominant kernel), with the same arguments and workspace.
 */
size_t cbf_lattice_workspace_size(int32_t W, int32_t win_rows, const cbf_grid* grid);

/* The nominal control the lattice builds form (a workspace setting, stream-ordered; a zero-filled
 * workspace holds CBF_NOMINAL_CONSENSUS).  CBF_NOMINAL_CONSENSUS: the lattice Laplacian scaled by
 * the call's gain (cross_and_rescue.py:121-125 shape).  CBF_NOMINAL_RANDOM: a synthetic random
 * walk, each component amp * (2 U - 1) with U in [0, 1) a hash of (seed, global agent index
 * win_row0 W + w, the bits of the agent's current position) -- fresh every step, identical under
 * any sharding (restated in oracle/pyoracle.py:random_nominal).  It keeps most QPs feasible with
 * a binding barrier row (the exact-QP regime); gain is then unused.  No reference counterpart:
 * cfg4 names a synthetic swarm, not its nominal controller. */
#define CBF_NOMINAL_CONSENSUS 0
#define CBF_NOMINAL_RANDOM 1
int cbf_lattice_set_nominal(void* workspace, size_t workspace_bytes, int32_t mode, double amp, uint64_t seed,
                            void* stream);

int cbf_lattice_step(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                     int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain, double T,
                     double* pos_out, double* vel_out, double* u, int32_t* status, int32_t* nbr_count,
                     int32_t guard_rows, double* extents, uint64_t* solves, void* workspace, size_t workspace_bytes,
                     void* stream);

/*
 * `steps` timesteps of a whole W x H lattice (rows [0, H), no halo) in one call: pos is advanced
 * in place; vel_out, u, status and nbr_count hold the last timestep's values; solves accumulates
 * over all of them.  Bit-identical to `steps` calls of cbf_lattice_step(p, grid, W, H, 0, H, 0, H,
 * pos, gain, T, pos, vel_out, u, status, nbr_count, 0, NULL, solves, ...) on the same workspace
 * (the reference's timestep loop, cross_and_rescue.py:97-175, run `steps` times).  Each advance
 * but the last bins the new positions for the next timestep's cell list as it writes them, so
 * the bin pass over all positions runs once per call instead of once per timestep.
 */
int cbf_lattice_run(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, double* pos, double gain,
                    double T, int32_t steps, double* vel_out, double* u, int32_t* status, int32_t* nbr_count,
                    uint64_t* solves, void* workspace, size_t workspace_bytes, void* stream);

/*
 * cbf_lattice_run with flags.  CBF_RUN_OUTPUT_HISTORY: vel_out, u, status and nbr_count are
 * arrays of `steps` timesteps (timestep t at element offset t W H of each) and every timestep's
 * values are stored -- the reference's per-step si_velocities (cross_and_rescue.py:159-160) for a
 * controller that consumes each step's filtered control.  flags = 0 is cbf_lattice_run.
 */
#define CBF_RUN_OUTPUT_HISTORY 1u
/* CBF_RUN_WINDOW_CULL: the lattice-window cull instead of the cell list (ABI 5).  Candidates come
 * straight from the lattice-ordered positions (the lattice neighbours of each ego), and per ego
 * two guards prove every agent it does not test out of cull range: row y-extents (suffix minima /
 * prefix maxima over rows) and per-row column x-extents.  Same neighbour sets, bit-identical
 * results; no cell-list build.  An ego whose neighbours are not lattice-near walks its rows
 * outward until the guards hold, so any swarm is handled exactly, the faster the more
 * lattice-like it stays (a consensus lattice: 5 rows x 3 columns of candidates; a scrambled one
 * degrades towards a whole-row scan -- use the cell list there).  Whole-lattice calls with
 * 4 <= W <= 2048; the grid argument still sizes and binds the workspace. */
#define CBF_RUN_WINDOW_CULL 2u
int cbf_lattice_run_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, double* pos, double gain,
                       double T, int32_t steps, double* vel_out, double* u, int32_t* status, int32_t* nbr_count,
                       uint64_t* solves, void* workspace, size_t workspace_bytes, uint32_t flags, void* stream);

/* The window-cull timestep in two calls, as cbf_lattice_build / cbf_lattice_advance_marked for the
 * cell list: the build (nominal control into vel_out and the workspace, the guards) and the
 * advance from the same pos into pos_out (which must not overlap pos), recording filter_done
 * (nullable hipEvent_t) between the filter kernel and the queued-QP kernel. */
/* The window cull's degradation counters of a lattice workspace, accumulated by every window-cull
 * advance since the workspace was zero-filled (statistics or not): out[0] = egos that took the
 * unbounded row walk, out[1] = row-guard words read at their spin limit.  Copied stream-ordered
 * into out (host or device memory, uint64[2]); synchronise the stream before reading a host copy.
 * A swarm that stops being lattice-like shows up here long before it shows in the timing; the cell
 * list (the same results) costs the same for any swarm.  (ABI 7) */
int cbf_lattice_window_counters(const void* workspace, size_t workspace_bytes, uint64_t* out, void* stream);

int cbf_lattice_window_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, const double* pos,
                             double gain, double* vel_out, void* workspace, size_t workspace_bytes, void* stream);
int cbf_lattice_window_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, const double* pos,
                               double T, double* pos_out, double* u, int32_t* status, int32_t* nbr_count,
                               uint64_t* stats, void* workspace, size_t workspace_bytes, void* filter_done,
                               void* stream);
/* The same for the owned rows [row_begin, row_end) of a window of win_rows lattice rows from
 * win_row0 (one sub-step of a sharded stripe); pos holds the window, pos_out the owned rows. */
int cbf_lattice_window_build_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                                double* vel_out, void* workspace, size_t workspace_bytes, void* stream);
int cbf_lattice_window_advance_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                  int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                                  double* pos_out, double* u, int32_t* status, int32_t* nbr_count, uint64_t* stats,
                                  void* workspace, size_t workspace_bytes, void* filter_done, void* stream);

int cbf_lattice_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                      int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                      double* vel_out, void* workspace, size_t workspace_bytes, void* stream);

int cbf_lattice_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                        int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                        double* pos_out, double* u, int32_t* status, int32_t* nbr_count, int32_t guard_rows,
                        double* extents, uint64_t* solves, void* workspace, size_t workspace_bytes, void* stream);

/* cbf_lattice_advance with Euclidean HOCBF rows (cbf_hocbf above): after cbf_lattice_build, the
 * filter of every owned agent over its 3x3-cell neighbours in ascending entity order, the HOCBF
 * QP, clip and Euler; same outputs, extents and solve counter as cbf_lattice_advance.  More than
 * 24 neighbours: CBF_STATUS_NBR_OVERFLOW (u = u0). */
/* Measurement hooks (the bench's timed launches of the filter kernel alone) are declared in
 * include/cbf_amd_measure.h: they are not part of the drop-in surface. */

int cbf_lattice_advance_hocbf(const cbf_params* p, const cbf_hocbf* hp, const cbf_grid* grid, int32_t W, int32_t H,
                              int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                              const double* pos, double T, double* pos_out, double* u, int32_t* status,
                              int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* solves,
                              void* workspace, size_t workspace_bytes, void* stream);

/*
 * Halo guard of the row-sharded lattice step.  ext_all holds world_size records of 4 doubles
 * (record q at ext_all + q * stride) as produced by cbf_lattice_step's `extents` with
 * guard_rows = halo - 1.  Sets *flag |= 1 (device int32) unless every agent outside rank's
 * candidate rows is farther than `radius` (in y) from every agent rank owns, i.e. unless the
 * halo exchange provably contained every neighbour.  One lane; stream-ordered.
 */
int cbf_halo_guard(const double* ext_all, int64_t stride, int32_t world_size, int32_t rank, double radius,
                   int32_t* flag, void* stream);

/*
 * Row-sharded step with ghost rows (what cbf_amd/shard.py runs).  A rank exchanges
 * every `nsub` sub-steps; each exchange is
 *   cbf_halo_pack -> all-gather of the send slabs (RCCL) -> cbf_halo_unpack,
 * and sub-step s then runs cbf_lattice_step_sharded on rows [row_begin, row_end) = the owned rows
 * widened by the ghost rows still exact at s, over the window of those rows +- the per-step halo.
 * cbf_lattice_step_sharded = cbf_lattice_step with solves counted over the owned rows
 * [own_begin, own_end) only, whose BUILD also accumulates y-extents of its INPUT positions into
 * ext_keys (sub-step s's set: ext_keys + s * cbf_halo_ext_bytes(1) / 8): {min, max over computed
 * rows, max over owned rows < own_end - guard_rows, min over owned rows >= own_begin +
 * guard_rows, min, max over owned rows}; guard_rows = the rows of a neighbour inside this
 * rank's candidate band at s.  The advance phase computes no extents.
 * cbf_halo_ext_bytes(nsub): size of nsub sets (512 slots x 16 uint64 keys each), set to identity
 * once with cbf_halo_ext_reset.  cbf_halo_pack writes send = [first `halo` owned rows | last
 * `halo` owned rows | nsub records of 8 doubles] (own = the n_own owned positions; halo = the
 * ghost depth) and resets the sets.  cbf_halo_unpack copies rank-1's last rows_lo rows into
 * window rows [0, rows_lo) and rank+1's first rows_hi rows into window rows [hi_row_offset,
 * +rows_hi) from the gathered recv (world_size slabs of `stride` doubles), and runs the halo guard
 * of every recorded sub-step: *flag |= 1 unless every agent outside a sub-step's candidate rows
 * was farther than the cull radius (in y) from every agent it computed.  The records describe the
 * sub-steps since the previous exchange, so a step is certified one exchange later (a final pack
 * + gather + unpack certifies the last ones).
 */
size_t cbf_halo_ext_bytes(int32_t nsub);
int cbf_halo_ext_reset(uint64_t* ext_keys, int32_t nsub, void* stream);
int cbf_halo_pack(int32_t W, int32_t halo, int64_t n_own, const double* own, uint64_t* ext_keys, int32_t nsub,
                  double* send, void* stream);
int cbf_halo_unpack(int32_t W, int32_t halo, int32_t rows_lo, int32_t rows_hi, int64_t hi_row_offset,
                    const double* recv, int64_t stride, int32_t world_size, int32_t rank, double radius, int32_t nsub,
                    double* wpos, int32_t* flag, void* stream);

/*
 * The neighbour form of the exchange (the default of cbf_amd/shard.py): ONE
 * all-to-all (RCCL all_to_all_single over xGMI) in which rank r sends its first `halo` owned rows to
 * r-1 only, its last `halo` rows to r+1 only, and its nsub guard records (8 doubles each) to every
 * rank.  Chunk q of send (to q) and of recv (from q), in rank order, is [nsub records | halo W
 * positions if q = r +- 1]; cbf_halo_nbr_elems gives the total doubles of either buffer (-1 on a
 * bad argument).  Per rank that is 2 halo W 16 B of rows instead of the all-gather's
 * world_size x that.  pack / unpack + guard as cbf_halo_pack / cbf_halo_unpack, same semantics.
 */
int64_t cbf_halo_nbr_elems(int32_t W, int32_t halo, int32_t nsub, int32_t world_size, int32_t rank);
int cbf_halo_pack_nbr(int32_t W, int32_t halo, int64_t n_own, const double* own, uint64_t* ext_keys, int32_t nsub,
                      int32_t world_size, int32_t rank, double* send, void* stream);
int cbf_halo_unpack_nbr(int32_t W, int32_t halo, int32_t rows_lo, int32_t rows_hi, int64_t hi_row_offset,
                        const double* recv, int32_t world_size, int32_t rank, double radius, int32_t nsub,
                        double* wpos, int32_t* flag, void* stream);
int cbf_lattice_step_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                             int32_t row_end, int32_t own_begin, int32_t own_end, int32_t win_row0, int32_t win_rows,
                             const double* pos, double gain, double T, double* pos_out, double* vel_out, double* u,
                             int32_t* status, int32_t* nbr_count, int32_t guard_rows, uint64_t* ext_keys,
                             uint64_t* solves, void* workspace, size_t workspace_bytes, void* stream);

/* One exchange cycle of the row-sharded step: the nsub sub-steps that follow the caller's
 * cbf_halo_unpack, bit-identical to nsub cbf_lattice_step_sharded calls with the geometry of
 * cbf_amd/shard.py (sub-step s computes rows [own_begin - d, own_end + d), d = halo (nsub - s - 1),
 * clamped to the lattice, over that band +- halo rows; guard rows d + halo - 1).  wpos and the
 * window-indexed outputs (wvel, wu, wstatus, wcnt nullable) cover rows [win_row0, win_row0 +
 * win_rows) = own +- halo nsub, clamped; ext_keys holds nsub extents sets (cbf_halo_ext_bytes);
 * workspaces holds nsub workspaces of ws_bytes >= cbf_lattice_workspace_size(W, win_rows, grid),
 * workspace s for sub-step s (kept across cycles).  Runs sub-steps [sub_begin, sub_end) of the
 * cycle (0 <= sub_begin < sub_end <= nsub; a whole cycle is [0, nsub)): the first of them bins
 * its window; every later sub-step's cell list is binned by the previous sub-step's advance as it
 * writes the rows.  The outputs of the call's last sub-step are written (its computed rows, which
 * contain the owned rows), as its cbf_lattice_step_sharded call would. */
int cbf_lattice_cycle_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t own_begin,
                              int32_t own_end, int32_t halo, int32_t nsub, int32_t sub_begin, int32_t sub_end,
                              int32_t win_row0, int32_t win_rows, double* wpos, double gain, double T, double* wvel,
                              double* wu, int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                              void* workspaces, size_t ws_bytes, void* stream);
/* cbf_lattice_cycle_sharded with flags: CBF_RUN_WINDOW_CULL runs every sub-step with the
 * lattice-window cull (workspaces as for the cell list; the call alternates between wpos and
 * workspace 0's sorted-position area, the last sub-step writing wpos).  Same results whenever the
 * halo guard holds. */
int cbf_lattice_cycle_sharded_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t own_begin,
                                 int32_t own_end, int32_t halo, int32_t nsub, int32_t sub_begin, int32_t sub_end,
                                 int32_t win_row0, int32_t win_rows, double* wpos, double gain, double T, double* wvel,
                                 double* wu, int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                                 void* workspaces, size_t ws_bytes, uint32_t flags, void* stream);

/*
 * Batched Monte-Carlo rendezvous (SURVEY cfg5): n_scen independent scenarios, each with
 * n_o pursuit obstacles (ring i -> i+1, rotation (rc, rs), scale so) then n_a free agents
 * (complete-graph consensus, gain ga; only they are filtered), `steps` Euler steps of T.
 * pos [n_scen][n_o + n_a][2] is updated in place.  counters [n_scen][4] int64 = {filter calls,
 * relaxed, box-infeasible, relax-cap}; maxviol [n_scen] = max row violation over the OPTIMAL
 * (feasible) solves; safety [n_scen][2] (nullable) = {max violation of the ORIGINAL barrier rows over
 * the RELAXED solves, min distance^2 from an agent to a culled neighbour (+inf if none)}.
 * maxviol may be NULL when safety is NULL: the kernel then computes no statistics (same positions
 * and counters).  One workgroup runs several scenarios for all steps with the state in LDS.
 * Requires 1 <= n_o, n_a and n_o + n_a <= 256.
 */
int cbf_mc_rollout(const cbf_params* p, int32_t n_scen, int32_t n_o, int32_t n_a, int32_t steps, double T, double rc,
                   double rs, double so, double ga, double* pos, int64_t* counters, double* maxviol, double* safety,
                   void* stream);

/*
 * robotarium-lite: the rps calls the reference scripts wrap around the
 * filter.  rps is third-party and absent (install.sh:1 clones it unpinned): these restate its
 * published algorithms; parity against rps itself is unpinned.
 *
 * Single-integrator barrier certificate with boundary -- replaces
 *   si_barrier_cert = create_single_integrator_barrier_certificate_with_boundary(safety_radius=0.12)
 *   si_velocities = si_barrier_cert(si_velocities, x_si[:, :4])      cross_and_rescue.py:72,163
 * (meet_at_center.py:58,109 creates it; its application is commented out there).  The coupled
 * QP  min |v - y|^2  s.t.  -2 e_ij.(v_i - v_j) <= gain h_ij^3 for every pair i < j and four
 * boundary rows per agent, y = dxi thresholded to magnitude_limit, is solved EXACTLY
 * (Goldfarb-Idnani dual active set; rps calls cvxopt.solvers.qp).  batch independent
 * scenarios of n_agents (1..32) each: dxi, x, out are [batch][n_agents][2] (agent-major: the
 * (2, N) rps arrays transposed).  status[batch] = CBF_CERT_*; iters / n_active may be NULL.
 * An infeasible QP (or the iteration cap) returns the thresholded input.
 */
#define CBF_CERT_OPTIMAL 1
#define CBF_CERT_INFEASIBLE 2
#define CBF_CERT_MAXITER 3
typedef struct cbf_cert_params {
    double barrier_gain;       /* 100 */
    double safety_radius;      /* 0.17 (cross_and_rescue.py:72 passes 0.12) */
    double magnitude_limit;    /* 0.2 */
    double boundary_points[4]; /* (-1.6, 1.6, -1.0, 1.0): x_min, x_max, y_min, y_max */
    double viol_tol;           /* a row counts as violated below -viol_tol * max(1, |b|) (1e-12) */
    int32_t max_iter;          /* 0 = 10 (m + 2 n_agents) + 10 */
} cbf_cert_params;
int cbf_cert_params_init(cbf_cert_params* c, double barrier_gain, double safety_radius, double magnitude_limit,
                         const double* boundary_points4);
size_t cbf_si_barrier_cert_lds_bytes(int32_t n_agents);
int cbf_si_barrier_cert(const cbf_cert_params* c, int32_t batch, int32_t n_agents, const double* dxi, const double* x,
                        double* out, int32_t* status, int32_t* iters, int32_t* n_active, void* stream);

/*
 * Unicycle side of the robotarium: poses are [n][3] = (x, y, theta) (the (3, N) rps array
 * transposed), single-integrator vectors [n][2].
 *   cbf_uni_to_si        uni_to_si_states (create_si_to_uni_mapping)  cross_and_rescue.py:75,101
 *   cbf_unicycle_advance mode 0: si_to_uni_dyn (:167) -> Robotarium.set_velocities (:170) ->
 *                        step (:175): motor (wheel-speed) threshold, Euler on (x, y, theta),
 *                        atan2 wrap; poses updated in place; dxu [n][2] = si_to_uni_dyn output
 *                        (may be NULL).  mode 1: si_to_uni_dyn alone (poses untouched, dxu
 *                        required).  mode 2: `dxi` holds unicycle (v, w): set_velocities + step.
 */
typedef struct cbf_unicycle_params {
    double projection_distance;    /* 0.05 */
    double angular_velocity_limit; /* pi (si_to_uni_dyn clamp) */
    double time_step;              /* 0.033 */
    double wheel_radius;           /* 0.016 */
    double base_length;            /* 0.105 */
    double max_linear_velocity;    /* 0.2 */
    double max_angular_velocity;   /* 2 (r / 0.11) (0.2 / r) */
    double max_wheel_velocity;     /* 0.2 / r */
    int32_t wheel_threshold;       /* 1: step() thresholds the wheel speeds */
} cbf_unicycle_params;
int cbf_unicycle_params_init(cbf_unicycle_params* u);
int cbf_uni_to_si(const cbf_unicycle_params* u, int32_t n, const double* poses, double* si, void* stream);
int cbf_unicycle_advance(const cbf_unicycle_params* u, int32_t n, double* poses, const double* dxi, double* dxu,
                         int32_t mode, void* stream);

/* ABI version of the loaded library (== CBF_ABI_VERSION). */
int cbf_abi_version(void);

/* Layout version of the lattice / cells workspaces (the control words, cell counts and starts, scan
 * tile words, sorted copies and queues a workspace holds between calls).  A saved workspace (e.g. a
 * rollout checkpoint) may be restored only into a library reporting the same version and size. */
int cbf_workspace_layout(void);

/* Byte offsets, inside a lattice workspace of this shape (cbf_lattice_workspace_size), of the cell
 * list the last cell-list build left (a diagnostic view for tests and tools; the kernels never need
 * it): off[0] start (int32[ncell + 1], the exclusive scan of the cell counts), off[1] the sorted
 * positions (double[n][2]), off[2] the sorted nominal controls, off[3] the sorted agent indices
 * (int32[n]); returns ncell, or CBF_EINVAL. */
int64_t cbf_lattice_workspace_view(int32_t W, int32_t win_rows, const cbf_grid* grid, int64_t* off);

#ifdef __cplusplus
}
#endif

#endif /* CBF_AMD_H */
