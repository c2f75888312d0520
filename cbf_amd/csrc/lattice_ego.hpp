// lattice_ego.hpp -- per-ego pieces shared by the lattice filters (swarm.hip: the cell-list cull,
// window.hip: the lattice-window cull): nominal controls, the solve / queue / output tail.
#pragma once

#include "cbf_device.hpp"
#include "cells.hpp"
#include "lattice.hpp"

namespace cbf {

constexpr int kExtSlotWords = 16;  // one 128-B line per extents slot (6 keys used)
constexpr int kExtSlots = 64;      // extents slots per sub-step set
constexpr int kExtVals = 6;        // {ego min, ego max, owned max below guard, owned min above guard, owned min, max}
__host__ __device__ constexpr bool ext_is_min(int q) { return q == 0 || q == 3 || q == 4; }

struct ExtSpec {
    int own_begin, own_end, guard;
};

// Halo-guard y-extents of one block's agents into slot (slot & (kExtSlots - 1)) of an extents
// set (e[] per lane: {min, max} over the computed rows, {max below the guard, min above it, min,
// max} over the owned rows; y = the lane's y where any).  The values travel as dkey()s (order-
// preserving uint64 keys, the form the slots hold), so each wave reduces them with 32-bit DPP
// reductions (wave_umin64 / wave_umax64) instead of 64-bit shuffle trees through LDS; a NaN y
// keys above +inf, so it wins a maximum and fails the guard (conservative).  The LAST wave of the
// block to arrive (an LDS counter, `arrive`, zeroed by the caller before a block barrier at
// kernel start) combines the NW partials and issues one atomic per non-identity value.  No
// barrier at the end (it would hold every wave until the block's slowest is done), and a quarter
// of the per-wave atomics.  ONE: each lane holds at most one agent (its e[] are y or infinite,
// which allows a two-reduction fast path).  Every lane of the wave must call it.
template <int NW>
__device__ __forceinline__ void ext_keys_combine(unsigned long long (&k)[6], unsigned long long* __restrict__ ext_keys,
                                                 long slot, unsigned long long (*red)[NW], int* arrive);
template <int NW, bool ONE = true>
__device__ __forceinline__ void ext_keys_flush(double (&e)[6], int any, double y,
                                               unsigned long long* __restrict__ ext_keys, long slot,
                                               unsigned long long (*red)[NW], int* arrive) {
    const unsigned long long kmin_id = dkey(INFINITY), kmax_id = dkey(-INFINITY);
    const unsigned long long act = __ballot(any);
    const unsigned code = any ? ((e[0] != INFINITY ? 1u : 0u) | (e[2] != -INFINITY ? 2u : 0u) |
                                 (e[3] != INFINITY ? 4u : 0u) | (e[4] != INFINITY ? 8u : 0u))
                              : 0u;
    const unsigned c0 = (unsigned)__shfl((int)code, act ? __ffsll((long long)act) - 1 : 0, 64);
    unsigned long long k[6];
    if (!act) {
#pragma unroll
        for (int q = 0; q < 6; ++q) k[q] = ext_is_min(q) ? kmin_id : kmax_id;
    } else if (ONE && __ballot(any && code != c0) == 0) {
        // the common wave: one membership pattern for all its agents, two reductions instead of six
        const unsigned long long ky = dkey(y);
        const unsigned long long mn = wave_umin64(any ? ky : kmin_id), mx = wave_umax64(any ? ky : kmax_id);
        k[0] = (c0 & 1u) ? mn : kmin_id;
        k[1] = (c0 & 1u) ? mx : kmax_id;
        k[2] = (c0 & 2u) ? mx : kmax_id;
        k[3] = (c0 & 4u) ? mn : kmin_id;
        k[4] = (c0 & 8u) ? mn : kmin_id;
        k[5] = (c0 & 8u) ? mx : kmax_id;
    } else {
#pragma unroll
        for (int q = 0; q < 6; ++q) k[q] = ext_is_min(q) ? wave_umin64(dkey(e[q])) : wave_umax64(dkey(e[q]));
    }
    ext_keys_combine<NW>(k, ext_keys, slot, red, arrive);
}

// The same for a block whose agents share one membership pattern (one lattice row: code bits
// 1 computed, 2 owned below the guard, 4 owned above it, 8 owned), from each lane's minimum lo
// (pmin) and maximum hi (NaN-propagating) over its agents: two wave reductions instead of six.
template <int NW>
__device__ __forceinline__ void ext_keys_flush_row(double lo, double hi, int any, unsigned code,
                                                   unsigned long long* __restrict__ ext_keys, long slot,
                                                   unsigned long long (*red)[NW], int* arrive) {
    const unsigned long long kmin_id = dkey(INFINITY), kmax_id = dkey(-INFINITY);
    const unsigned long long mn = wave_umin64(any ? dkey(lo) : kmin_id), mx = wave_umax64(any ? dkey(hi) : kmax_id);
    unsigned long long k[6];
    k[0] = (code & 1u) ? mn : kmin_id;
    k[1] = (code & 1u) ? mx : kmax_id;
    k[2] = (code & 2u) ? mx : kmax_id;
    k[3] = (code & 4u) ? mn : kmin_id;
    k[4] = (code & 8u) ? mn : kmin_id;
    k[5] = (code & 8u) ? mx : kmax_id;
    ext_keys_combine<NW>(k, ext_keys, slot, red, arrive);
}

// the block-level half of the flushes: the last wave to arrive combines the partials and issues
// one atomic per non-identity value
template <int NW>
__device__ __forceinline__ void ext_keys_combine(unsigned long long (&k)[6], unsigned long long* __restrict__ ext_keys,
                                                 long slot, unsigned long long (*red)[NW], int* arrive) {
    const unsigned long long kmin_id = dkey(INFINITY), kmax_id = dkey(-INFINITY);
    if ((threadIdx.x & 63) != 0) return;
    const int wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 6; ++q) red[q][wid] = k[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (atomicAdd(arrive, 1) != NW - 1) return;  // not the last wave of the block
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int v = 0; v < NW; ++v)
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const unsigned long long x = red[q][v];
            k[q] = ext_is_min(q) ? (x < k[q] ? x : k[q]) : (x > k[q] ? x : k[q]);
        }
    unsigned long long* ks = ext_keys + kExtSlotWords * (slot & (kExtSlots - 1));
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        if (ext_is_min(q)) {
            if (k[q] != kmin_id) atomicMin(&ks[q], k[q]);
        } else if (k[q] != kmax_id) {
            atomicMax(&ks[q], k[q]);
        }
    }
}


// Lattice Laplacian sum for window agent w (neighbours in ascending index order).
__device__ __forceinline__ double2 lattice_sum(const double2* __restrict__ pos, long w, int r, int c, int W, int H) {
    const double2 pi = pos[w];
    double a0 = 0.0, a1 = 0.0;
    if (r > 0) {
        const double2 q = pos[w - W];
        a0 = a0 + (q.x - pi.x);
        a1 = a1 + (q.y - pi.y);
    }
    if (c > 0) {
        const double2 q = pos[w - 1];
        a0 = a0 + (q.x - pi.x);
        a1 = a1 + (q.y - pi.y);
    }
    if (c < W - 1) {
        const double2 q = pos[w + 1];
        a0 = a0 + (q.x - pi.x);
        a1 = a1 + (q.y - pi.y);
    }
    if (r < H - 1) {
        const double2 q = pos[w + W];
        a0 = a0 + (q.x - pi.x);
        a1 = a1 + (q.y - pi.y);
    }
    return make_double2(a0, a1);
}

// CBF_NOMINAL_RANDOM: a random-walk nominal control, a pure function of (seed, global agent
// index, the bits of the agent's current position): splitmix64 finalisers chained over the three
// words; each component amp (2 U - 1) with U = (h >> 11) 2^-53 (2 U - 1 is exact, so the only
// rounding is the product).  The position changes every step, so each step draws afresh, with no
// step counter; any sharding of the lattice draws the same values.  Restated in
// oracle/pyoracle.py:random_nominal.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double2 random_nominal(const NominalSpec& N, long g, double2 p) {
    unsigned long long h = mix64(N.seed + 0x9E3779B97F4A7C15ull * (unsigned long long)(g + 1));
    h = mix64(h ^ (unsigned long long)__double_as_longlong(p.x));
    h = mix64(h ^ (unsigned long long)__double_as_longlong(p.y));
    const unsigned long long h2 = mix64(h + 0x9E3779B97F4A7C15ull);
    const double v0 = 2.0 * ((double)(h >> 11) * 0x1p-53) - 1.0;
    const double v1 = 2.0 * ((double)(h2 >> 11) * 0x1p-53) - 1.0;
    return make_double2(N.amp * v0, N.amp * v1);
}

// Per-ego outcome of the lattice filter for the statistics.
struct EgoOut {
    int res;          // 0 not an owned ego, 1 done (outputs written), 2 queued for the full solve
    int w;            // window index of the agent
    int nbrs;         // neighbours
    int code;         // final status code (res == 1)
    bool binding;     // the minimiser is not the origin (res == 1)
    bool seidel;      // the QP took the full Seidel solve (inline, or through the queue)
    double viol, vorig, d2, nx, ny;
};

// Where the QPs that solve_fast cannot settle are solved: windows of at most
// cbf_params.solve_inline_max agents (a runtime setting; < 0 = kSolveInlineDefault) run the filter
// instantiation with the full solve inline (IN = true: no queue kernel); larger ones queue the QPs
// with their assembled state for k_lattice_filter_hard, one lane per QP.  Measured crossover
// (cbf_lattice_run, W = 1024, spacing 0.145, run(10) per timestep, inline vs queue): 64 rows 25.2 vs
// 30.2 us, 128 rows 27.7 vs 32.6 us, 256 rows 42.5 vs 38.9 us, 512 rows 55 vs 55 (and the inline
// form at 1024 rows 118.5 vs 79.5).  Between 128 and 192 rows (tools/records/gpu_r03g2.sh): 128 rows
// 27.8-27.9 vs 32.5-32.7, 136 rows 34.2 vs 32.9-33.1, 144 35.0 vs 33.8, 160 35.6 vs 33.8, 192
// 38.5-38.8 vs 34.0-34.6.  So the inline form pays only while every SIMD holds at most 2 of the
// window's waves: 256 CUs x 4 SIMDs x 2 waves x 64 lanes = 131072 agents (one 1024-wide row more
// puts a third 165-VGPR wave on some SIMDs, and the kernel ends with the most loaded one).  The two
// placements are bit-identical (tests run both).  The wave-cooperative solves measured slower in
// either place: commit c7a6b09 and branch exp/coop-line-solve.
constexpr long kSolveInlineDefault = 131072;
inline bool solve_inline(const cbf_params* p, long n) {
    return n <= (p->solve_inline_max < 0 ? kSolveInlineDefault : (long)p->solve_inline_max);
}

// Outputs of one owned ego (output index k) once its QP is solved (or it has no neighbour):
// clip, Euler, stores, statistics record.
template <bool ST>
__device__ __forceinline__ void ego_output(const KP& P, const Ego& E, const Sol& S, bool idle, int k, double T,
                                           double2* __restrict__ pos_out, double2* __restrict__ u,
                                           int32_t* __restrict__ status, int32_t* __restrict__ cnt, EgoOut& O) {
    double ux, uy;
    int32_t st;
    O.code = CBF_STATUS_IDLE;
    if (idle) {
        ux = E.u0x;
        uy = E.u0y;
        st = CBF_STATUS_IDLE;
    } else {
        clip_u(P, S, E, ux, uy);
        st = pack_status(S);
        O.code = S.status;
        if (ST) {  // statistics only (a kernel without them compiles the violations away)
            O.binding = S.x0 != 0.0 || S.x1 != 0.0;
            O.viol = S.viol;
            O.vorig = S.viol_orig;
        }
    }
    const double2 pn = make_double2(E.r0 + T * ux, E.r1 + T * uy);
    st_stream(pos_out + k, pn);
    if (u) u[k] = make_double2(ux, uy);  // u / status / cnt: null in the inner timesteps of cbf_lattice_run
    if (status) status[k] = st;
    if (cnt) cnt[k] = E.count;
    O.nx = pn.x;
    O.ny = pn.y;
    O.res = 1;
}

// Tail of the lattice filter for one owned ego (output index k) whose QP rows are accumulated in
// E.  IN (the small-window instantiation): solve in place when solve_fast can (origin, or one
// Seidel event that stays put), else run the full solve_ego right here.  Queued form: settle the
// origin case here and queue every other QP to the hard kernel (sub-queue q: header hardq, records
// qrec, subq_append).  Then clip, Euler, outputs.
#ifndef CBF_EVENT_IN_PLACE
#define CBF_EVENT_IN_PLACE 8
#endif
constexpr int kEventInPlace = CBF_EVENT_IN_PLACE;
template <bool FZ, bool ST, bool IN>
__device__ __forceinline__ void ego_finish(const KP& P, Ego& E, int w, int k, int slot, double T,
                                           double2* __restrict__ pos_out, double2* __restrict__ u,
                                           int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                           int32_t* __restrict__ hardq, int q, HardRec* __restrict__ qrec,
                                           long qcap, EgoOut& O) {
    Sol S;
    const bool idle = E.count == 0;
    // The queued form runs solve_fast's one-event stage only in a wave where more than
    // kEventInPlace lanes need it; the others' QPs go to the queue kernel whole, so that no filter
    // wave runs the event stage for one lane (cfg4: 0.5 % of the egos, about one per wave), while
    // a regime where most QPs take one event (cfg4f) does not move them all to the queue.  run(10)
    // per timestep at 1 M agents, window cull, cfg4 / cfg4f: 63.7 / 59.2 us without deferral;
    // threshold 4: 62.8 / 59.6; 8: 62.3 / 60.1; every event queued: 61.9 / 69.2.  The inline form
    // (small windows, no queue kernel) keeps the one-event stage for every lane.
    FastState F;
    bool done = idle;
    if (!done) done = IN ? solve_fast(P, E, S) : fast_origin(P, E, F, S);
    if (!IN && !done && __popcll(__ballot(1)) > kEventInPlace) done = fast_event(P, E, F, S);
    if (!done) {
        O.seidel = IN;  // (queued: the queue kernel counts the QPs solve_fast cannot settle)
        if (IN) {
            S = solve_ego(P, E);
            ego_output<ST>(P, E, S, false, k, T, pos_out, u, status, cnt, O);
            return;
        }
        const long rec = subq_append(hardq, q, qcap);
        O.res = 2;
        if (rec < 0) return;  // (unreachable: the queue holds every agent and is emptied every advance)
        HardRec& h = qrec[rec];
        h.r0 = E.r0;
        h.r1 = E.r1;
        h.r2 = E.r2;
        h.r3 = E.r3;
        h.u0x = E.u0x;
        h.u0y = E.u0y;
        h.bq0 = E.bq0;
        h.bq1 = E.bq1;
        h.bq2 = E.bq2;
        h.bq3 = E.bq3;
        h.present = (int)E.present;
        h.count = E.count;
        h.k = k;
        h.row = w;
        h.slot = slot;
        return;
    }
    ego_output<ST>(P, E, S, idle, k, T, pos_out, u, status, cnt, O);
}

// The lattice-window cull (window.hip, CBF_RUN_WINDOW_CULL).  Geometry of a call: arrays of `rows`
// lattice rows from lattice row row0 of a W x Hl lattice, candidates in window rows [cr0, cr1).
struct WinGeom {
    int W, rows, row0, Hl, cr0, cr1;
};
inline WinGeom whole_lattice(int W, int H) { return WinGeom{W, H, 0, H, 0, H}; }
// whether a call of this geometry can use it (rows of 4 .. 2048 agents, guard arrays in the
// workspace's record area)
bool window_cull_ok(int W, int rows, long n_ws, const CellWs& Wk);
// The build: nominal controls (vel_out: index (r - row_begin) W + c for rows [row_begin, row_end),
// nullable), the guards, the halo-guard extents (ext_keys, nullable: sharded), a copy of pos
// (copy_to, nullable).
// the window cull's row guard formed inside the filter launch (else by a separate scan kernel
// launched with the build): cbf_params.launch_flags
bool window_fold(const cbf_params* p);
int window_counters(const void* workspace, size_t workspace_bytes, uint64_t* out, hipStream_t s);
void window_prep(const CellWs& Wk, const WinGeom& Q, const double2* pos, double gain, double2* vel_out,
                 double2* copy_to, unsigned long long* ext_keys, int row_begin, int row_end, ExtSpec X,
                 bool fold, hipStream_t s);
// The filter kernel for the egos of lattice rows [row_begin, row_end) (pos_out must not overlap pos;
// the queued QPs are left for k_lattice_filter_hard unless `in`).
void window_filter(const cbf_params* p, const CellWs& Wk, const WinGeom& Q, int row_begin, int row_end,
                   int cnt_begin, int cnt_end, const double2* pos, double T, double2* pos_out, double2* u,
                   int32_t* status, int32_t* cnt, unsigned long long* stats, bool in, hipStream_t s,
                   hipEvent_t t_start = nullptr, hipEvent_t t_stop = nullptr);

}  // namespace cbf
