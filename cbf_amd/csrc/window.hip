// window.hip -- the lattice-window cull of a lattice swarm timestep (gfx950).
//
// The cull of cross_and_rescue.py:141-150 keeps, for each ego, the agents within the cull radius.
// The cell-list path (swarm.hip) finds them through a counting sort of all positions by cell,
// rebuilt every timestep.  An agent of a lattice swarm keeps its lattice index, and while the
// swarm stays lattice-like its neighbours are lattice neighbours: this path takes the candidates
// straight from the lattice-ordered positions (coalesced loads, no sort) and PROVES per ego that
// every agent it does not test is out of range, so the neighbour sets -- and every result -- are
// bit-identical to the cell-list path's (the per-quadrant minimum is order-independent).
//
// The proof uses two guards, both exact in fp64 (rounding is monotone, so a computed difference
// beyond d = win_d makes e * e >= cull_t: the candidate fails s < cull_t):
//   rows     per lattice row the min / max y over its agents; sylo[r] = min over rows >= r,
//            pyhi[r] = max over rows <= r (formed by the filter launch's first block).  Rows
//            r + k + 1 and beyond are out of range of an ego at y once sylo[r + k + 1] - y > d
//            (and below likewise).
//   columns  per agent of row r' the min x over the columns >= its own (rs) and the max x over the
//            columns <= its own (rp), rounded outward to fp32.  Columns c' and beyond of row r'
//            are out of range once rs(r', c') - x > d (and to the left likewise).
// Agents with a non-finite coordinate can never pass the cull test and are left out of every
// extent.  The filter (k_window_tile) stages a tile of rows and its halo in LDS; each ego scans
// its rows (the row guard, up to -+3) over columns c - 1 .. c + 1 and checks the column sentinels
// at c -+ 2; a wave whose lanes need it scans columns c -+ 2 too (sentinels at c -+ 3); a lane
// that still needs more walks its rows outward until every sentinel holds, with direct row
// assembly (win_direct: any swarm, slower the less lattice-like it is).
#include <hip/hip_ext.h>
#include "cbf_device.hpp"
#include "cells.hpp"
#include "lattice.hpp"
#include "lattice_ego.hpp"

using namespace cbf;

extern "C" __device__ __attribute__((const)) double __ockl_wfred_min_f64(double);
extern "C" __device__ __attribute__((const)) double __ockl_wfred_max_f64(double);

namespace {

#ifndef CBF_TILE_EARLY_ROWS
#define CBF_TILE_EARLY_ROWS 1  // rows -1..+1 tested before the row guard is read (0: after)
#endif
#ifndef CBF_TILE_FUSED_FLUSH
#define CBF_TILE_FUSED_FLUSH 1  // 0: the hits' rows formed after the scan, from the hit mask (round 6)
#endif
#ifndef CBF_TILE_WPE
#define CBF_TILE_WPE 6  // waves per SIMD the timed tile kernels (queued solve, no statistics) are fitted to
#endif
#ifndef CBF_GUARD_PER
#define CBF_GUARD_PER 2  // rows per thread of the tile launch's row-guard scan
#endif
#ifndef CBF_WIN_SPIN_LIMIT
#define CBF_WIN_SPIN_LIMIT (1l << 22)  // polls of a row-guard word before it reads as the worst bound
#endif
#ifndef CBF_PREP_BLOCK
#define CBF_PREP_BLOCK 256  // threads of a build block (one lattice row)
#endif
#ifndef CBF_PREP_WPE
#define CBF_PREP_WPE 1  // waves per SIMD the build kernel's registers are fitted to (1: no fit)
#endif
constexpr int kPrepBlock = CBF_PREP_BLOCK;
constexpr int kPrepWideRows = 256;  // windows of at most this many rows: 2 kPrepBlock threads per row
constexpr int kWinMaxW = 2048;                  // rows of up to 2048 agents

// The guard arrays in the workspace's record area (cs, 16 B per agent, unused by this path).
struct WinGuard {
    double* rowy;     // [2 H] {min y, max y} per row (finite agents)
    double* sylo;     // [H + 1] min over rows >= r of the row minima (sylo[H] = +inf)
    double* pyhi;     // [H] max over rows <= r of the row maxima
    int32_t* srt;     // [H] 1: every agent of the row finite and x non-decreasing along it (then each
                      // agent's own x is its column extents, and the build stores none for the row)
};
inline WinGuard win_guard(const CellWs& Wk, int H) {
    WinGuard g;
    char* p = reinterpret_cast<char*>(Wk.cs);
    g.rowy = reinterpret_cast<double*>(p);
    g.sylo = g.rowy + 2l * H;
    g.pyhi = g.sylo + (H + 1);
    g.srt = reinterpret_cast<int32_t*>(g.pyhi + H);
    return g;
}
// Control words of the window cull in the workspace header (fixed offsets, whatever the lattice
// shape or the cull another call used on the workspace; cells.hpp CellWs::sctl):
//   sctl[kWinTokenWord]  the guard-token count, advanced by every window build;
//   sctl[kWinModeWord]   how the last build's row guard is formed: kGuardInFilter (the filter
//                        launch's first block forms it as token-tagged words) or kGuardSeparate
//                        (k_window_rowscan wrote plain doubles).  The filter follows this word,
//                        not its own cbf_params, so a build and an advance that disagree on
//                        CBF_LAUNCH_SEPARATE_GUARD still read the guard the build prepared.
//   sctl[kWinWalkWord]   (uint64) egos that took the unbounded walk (win_direct), and
//   sctl[kWinStallWord]  (uint64) row-guard words read at their spin limit (as the worst bound),
//                        both accumulated by every window filter since the workspace was zero-filled
//                        (cbf_lattice_window_counters): the cull stays exact either way, these say
//                        how far it has degraded from its lattice-neighbour fast path.
constexpr int kWinTokenWord = 16, kWinModeWord = 17, kWinWalkWord = 20, kWinStallWord = 22;
constexpr int32_t kGuardInFilter = 1, kGuardSeparate = 2;
// a build's guard token: a 24-bit count tagged in the top byte (the guard area is the cell list's
// record area on other paths; its words never carry the tag).  The count lives in the header, so
// tokens keep increasing across culls and lattice shapes sharing a workspace.
__host__ __device__ inline int32_t guard_token(int32_t v) { return (v & 0x00FFFFFF) | 0x5A000000; }
inline size_t win_guard_bytes(int H) { return 8 * (size_t)(4l * H + 2) + 4 * (size_t)H; }  // <= 16 W H for W >= 4
// Geometry (WinGeom, lattice_ego.hpp): candidates are the agents of window rows [cr0, cr1).  A
// window edge that is not a lattice edge is not a candidate row (its agents' nominal controls
// cannot be formed there; the cell-list builds skip them likewise, and the sharded step's halo
// guard proves them out of range), so for the guards rows beyond [cr0, cr1) do not exist.

// the column extents, one float2 {rs, rp} per agent, in the scratch area (wvel, 16 B per agent)
inline float2* win_rsp(const CellWs& Wk) { return reinterpret_cast<float2*>(Wk.wvel); }

// fp32 bounds of a double: the largest float <= v / the smallest float >= v (outward rounding, so
// the column guard built from them stays sound)
__device__ __forceinline__ float f32_down(double v) {
    float f = (float)v;
    if ((double)f > v) {
        const unsigned b = __float_as_uint(f);
        f = f == 0.0f ? __uint_as_float(0x80000001u) : __uint_as_float(f > 0.0f ? b - 1u : b + 1u);
    }
    return f;
}
__device__ __forceinline__ float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) {
        const unsigned b = __float_as_uint(f);
        f = f == 0.0f ? __uint_as_float(0x00000001u) : __uint_as_float(f > 0.0f ? b + 1u : b - 1u);
    }
    return f;
}

// Minima / maxima of guard extents: the values are finite or +-inf (non-finite agents are left
// out), never NaN, and the sign of a zero cannot change a guard test (d > 0), so the min / max
// instruction serves as is: one VALU op instead of pmin's compare and two selects (fmin would
// add the IEEE-mode quieting of each operand).
__device__ __forceinline__ double gmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double gmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Window-cull build of one timestep: one block per candidate row.  Per agent the nominal control
// (the lattice Laplacian of cross_and_rescue.py:121-125 shape scaled by gain, or the random walk
// of CBF_NOMINAL_RANDOM: the scatter's arithmetic) into u0 (and vel_out), the column extents into
// rsp; per row its y extents (turned into the row guard by the filter launch); the sharded step's
// halo-guard extents (ext_keys, nullable).  copy_to (nullable) gets a copy of the positions (the
// run's ping-pong start).  The row is staged in LDS (dynamic, 24 B per column): every global load
// and store is coalesced, and the row scans run over contiguous chunks of it.
template <int PER, int NT>  // columns per thread (W <= NT x PER), threads of the block
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(CBF_PREP_WPE))) k_window_prep(WinGeom Q, const double2* __restrict__ pos,
                                                            double2* __restrict__ u0, float2* __restrict__ rsp,
                                                            WinGuard Gd, double gain, double2* __restrict__ vel_out,
                                                            double2* __restrict__ copy_to, int32_t* __restrict__ sctl,
                                                            long ncell, unsigned long long* __restrict__ ext_keys,
                                                            int row_begin, int row_end, ExtSpec X, int32_t guard_mode) {
    extern __shared__ double2 srow[];  // [W] positions, then [W] float2 {rs, rp}
    const int W = Q.W;
    float2* srsp = reinterpret_cast<float2*>(srow + W);
    __shared__ double red4[4][NT / 64];
    __shared__ unsigned long long ered[6][NT / 64];
    __shared__ int arrive;
    const int r = Q.cr0 + xcd_block();      // window row
    const int rl = Q.row0 + r;              // lattice row
    const long nwin = (long)W * Q.rows;
    if (r == Q.cr0 && threadIdx.x == 0) {
        build_begin(sctl, nwin, ncell);
        sctl[kWinTokenWord] = (sctl[kWinTokenWord] + 1) & 0x00FFFFFF;  // this build's guard token
        sctl[kWinModeWord] = guard_mode;
    }
    if (ext_keys && threadIdx.x == 0) arrive = 0;
    const NominalSpec N = nominal_spec(sctl);
    const bool lap = N.mode != CBF_NOMINAL_RANDOM;
    const double2* prow = pos + (long)r * W;
    // every load of the block in one round trip: the row (coalesced: column c = thread + j * block)
    // and, for the Laplacian, the rows above and below
    double2 p[PER], qu[PER], qd[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * NT;
        if (c < W) {
            p[j] = prow[c];
            if (lap && rl > 0) qu[j] = prow[c - W];
            if (lap && rl < Q.Hl - 1) qd[j] = prow[c + W];
        }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * NT;
        if (c < W) {
            srow[c] = p[j];
            if (copy_to) copy_to[(long)r * W + c] = p[j];
        }
    }
    __syncthreads();
    // nominal controls and the row's y extents: every column's value first, then all the stores
    // together, so that no later wait for a load result also waits for a store in flight (a wait
    // between the columns' stores serialised their round trips: 11.8 against 8.8 us per build at
    // 1 M agents)
    double ylo = INFINITY, yhi = -INFINITY;
    double2 a[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * NT;
        const double2 pi = p[j];
        if (!lap) {
            a[j] = random_nominal(N, (long)Q.row0 * W + (long)r * W + c, pi);
        } else {  // lattice_sum's neighbour order and arithmetic: (r-1, c), (r, c-1), (r, c+1), (r+1, c)
            double a0 = 0.0, a1 = 0.0;
            if (rl > 0) {
                a0 = a0 + (qu[j].x - pi.x);
                a1 = a1 + (qu[j].y - pi.y);
            }
            if (c > 0) {
                const double2 q = srow[c - 1];
                a0 = a0 + (q.x - pi.x);
                a1 = a1 + (q.y - pi.y);
            }
            if (c < W - 1) {
                const double2 q = srow[c + 1];
                a0 = a0 + (q.x - pi.x);
                a1 = a1 + (q.y - pi.y);
            }
            if (rl < Q.Hl - 1) {
                a0 = a0 + (qd[j].x - pi.x);
                a1 = a1 + (qd[j].y - pi.y);
            }
            a[j] = make_double2(a0 * gain, a1 * gain);
        }
        const bool f = c < W && isfinite(pi.x) && isfinite(pi.y);  // (a column beyond W: no agent)
        const double lo = gmin(ylo, pi.y), hi = gmax(yhi, pi.y);
        ylo = f ? lo : ylo;
        yhi = f ? hi : yhi;
    }
    const bool vo = vel_out && rl >= row_begin && rl < row_end;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * NT;
        if (c >= W) continue;
        st_stream(u0 + (long)r * W + c, a[j]);
        if (vo) vel_out[(long)(rl - row_begin) * W + c] = a[j];
    }
    // A sorted row (every agent finite, x non-decreasing along it: a lattice row under consensus)
    // needs no column extents -- each agent's own x is the minimum over the columns from it on and
    // the maximum over those up to it -- so the filter reads the staged positions instead and the
    // build skips the scans and the 8-B store per agent.  Other rows: suffix minimum / prefix
    // maximum of x over the finite agents, each thread over its contiguous chunk of m columns, then
    // across the threads, through one block-wide exchange with the row's y extents.
    bool ok = true;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * NT;
        if (c < W) {
            ok = ok && isfinite(p[j].x) && isfinite(p[j].y);
            if (c + 1 < W) ok = ok && p[j].x <= srow[c + 1].x;
        }
    }
    // block-wide AND: a vote per wave, one barrier (__syncthreads_and took three and LDS atomics:
    // 11.1 against 11.5 us per build at 1 M agents)
    __shared__ int s_ok[NT / 64];
    {
        const bool wok = __all(ok) != 0;
        if ((threadIdx.x & 63) == 0) s_ok[threadIdx.x >> 6] = wok ? 1 : 0;
    }
    __syncthreads();
    bool sorted = true;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) sorted = sorted && s_ok[q] != 0;
    const int m = (W + NT - 1) / NT;
    const int c0 = threadIdx.x * m;
    double sm[PER], pm[PER];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double ss = INFINITY, ps = -INFINITY, yl = ylo, yh = yhi;  // wave scans / reductions
    if (!sorted) {
        double acc = INFINITY;
#pragma unroll
        for (int j = PER - 1; j >= 0; --j) {
            if (j < m && c0 + j < W) {
                const double2 q = srow[c0 + j];
                if (isfinite(q.x) && isfinite(q.y)) acc = gmin(acc, q.x);
            }
            sm[j] = acc;
        }
        acc = -INFINITY;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (j < m && c0 + j < W) {
                const double2 q = srow[c0 + j];
                if (isfinite(q.x) && isfinite(q.y)) acc = gmax(acc, q.x);
            }
            pm[j] = acc;
        }
        ss = sm[0];
        ps = pm[PER - 1];
        for (int o = 1; o < 64; o <<= 1) {
            const double a = __shfl_down(ss, o, 64), b = __shfl_up(ps, o, 64);
            if (lane + o < 64) ss = gmin(ss, a);
            if (lane >= o) ps = gmax(ps, b);
        }
    }
    yl = __ockl_wfred_min_f64(yl);  // DPP wave reductions (the extents are finite or +-inf)
    yh = __ockl_wfred_max_f64(yh);
    double sx = __shfl_down(ss, 1, 64), px = __shfl_up(ps, 1, 64);  // exclusive
    if (lane == 63) sx = INFINITY;
    if (lane == 0) px = -INFINITY;
    if (lane == 0) red4[0][wid] = ss;
    if (lane == 63) red4[1][wid] = ps;
    if (lane == 0) {
        red4[2][wid] = yl;
        red4[3][wid] = yh;
    }
    __syncthreads();
    double after = sx, before = px, lo = INFINITY, hi = -INFINITY;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) {
        if (q > wid) after = gmin(after, red4[0][q]);
        if (q < wid) before = gmax(before, red4[1][q]);
        lo = gmin(lo, red4[2][q]);
        hi = gmax(hi, red4[3][q]);
    }
    if (!sorted) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = c0 + j;
            if (j < m && c < W) srsp[c] = make_float2(f32_down(gmin(sm[j], after)), f32_up(gmax(pm[j], before)));
        }
    }
    if (ext_keys) {
        // the sharded step's halo-guard extents of this build's input positions (as the cell-list
        // bin kernel accumulates them, every agent of the row, non-finite ones included): {min,
        // max} over the computed rows, {max below the guard, min above it, min, max} over the owned
        // (the membership is the row's: each thread's minimum and maximum over its columns, then
        // two wave reductions)
        auto nmax = [](double mm, double y) { return (y > mm || y != y) ? y : mm; };
        const bool comp = rl >= row_begin && rl < row_end, own = rl >= X.own_begin && rl < X.own_end;
        const unsigned code = (comp ? 1u : 0u) | (own && rl < X.own_end - X.guard ? 2u : 0u) |
                              (own && rl >= X.own_begin + X.guard ? 4u : 0u) | (own ? 8u : 0u);
        double elo = INFINITY, ehi = -INFINITY;  // (not the row's y extents lo / hi the row guard stores)
        int any = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = threadIdx.x + j * NT;
            if (c >= W) continue;
            elo = pmin(elo, p[j].y);
            ehi = nmax(ehi, p[j].y);
            any = 1;
        }
        ext_keys_flush_row<NT / 64>(elo, ehi, any && code != 0u, code, ext_keys, r, ered, &arrive);
    }
    if (!sorted) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = threadIdx.x + j * NT;
            if (c < W) rsp[(long)r * W + c] = srsp[c];
        }
    }
    if (threadIdx.x == 0) {
        Gd.rowy[2l * r] = lo;
        Gd.rowy[2l * r + 1] = hi;
        Gd.srt[r] = sorted ? 1 : 0;
    }
}

// The row guard's arrays from the row extents k_window_prep wrote (one block, one row per thread
// and chunk): sylo[r] = min over candidate rows >= r of the row minima (sylo[cr1] = +inf),
// pyhi[r] = max over candidate rows <= r of the row maxima.  (A ticket at the end of the prep
// kernel, whose last block did this, serialised 1,024 same-address atomics: 29 us per build.)
constexpr int kRowScanBlock = 1024;
template <bool PACK>  // PACK: {fp32 value, token} words (in-launch hand-off), else the double
__device__ __forceinline__ void st_guard(double* p, double v, bool down, int32_t token) {
    if (PACK) {
        const float f = down ? f32_down(v) : f32_up(v);
        const unsigned long long w = ((unsigned long long)(uint32_t)token << 32) | __float_as_uint(f);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *p = v;
    }
}
template <int NT, int PER, bool PACK>  // threads of the block, rows per thread and chunk
__device__ __forceinline__ void row_guard_scan(const WinGeom& Q, const WinGuard& Gd, double (*red)[NT / 64],
                                               int32_t token) {
    constexpr int NW = NT / 64, CH = NT * PER;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int lo = Q.cr0, H = Q.cr1;
    // chunks of PER consecutive rows per thread (all loads of a chunk in one round trip); suffix
    // minima run from the last chunk down, prefix maxima up
    double carry_s = INFINITY, carry_p = -INFINITY;
    const int nch = (H - lo + CH - 1) / CH;
    for (int k = 0; k < nch; ++k) {
        const int bs = lo + (nch - 1 - k) * CH + threadIdx.x * PER;  // suffix pass rows bs .. bs + PER - 1
        const int bp = lo + k * CH + threadIdx.x * PER;              // prefix pass rows
        double ls[PER], lp[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            ls[j] = bs + j < H ? Gd.rowy[2l * (bs + j)] : INFINITY;
            lp[j] = bp + j < H ? Gd.rowy[2l * (bp + j) + 1] : -INFINITY;
        }
#pragma unroll
        for (int j = PER - 2; j >= 0; --j) ls[j] = gmin(ls[j], ls[j + 1]);
#pragma unroll
        for (int j = 1; j < PER; ++j) lp[j] = gmax(lp[j], lp[j - 1]);
        double vs = ls[0], vp = lp[PER - 1];
        for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scans of the thread totals
            const double a = __shfl_down(vs, o, 64), b = __shfl_up(vp, o, 64);
            if (lane + o < 64) vs = gmin(vs, a);
            if (lane >= o) vp = gmax(vp, b);
        }
        double xs = __shfl_down(vs, 1, 64), xp = __shfl_up(vp, 1, 64);  // exclusive
        if (lane == 63) xs = INFINITY;
        if (lane == 0) xp = -INFINITY;
        if (lane == 0) red[0][wid] = vs;
        if (lane == 63) red[1][wid] = vp;
        __syncthreads();
        double as = carry_s, bq = carry_p, ts = INFINITY, tp = -INFINITY;
        for (int q = 0; q < NW; ++q) {
            if (q > wid) as = gmin(as, red[0][q]);
            if (q < wid) bq = gmax(bq, red[1][q]);
            ts = gmin(ts, red[0][q]);
            tp = gmax(tp, red[1][q]);
        }
        as = gmin(as, xs);
        bq = gmax(bq, xp);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (bs + j < H) st_guard<PACK>(&Gd.sylo[bs + j], gmin(ls[j], as), true, token);
            if (bp + j < H) st_guard<PACK>(&Gd.pyhi[bp + j], gmax(lp[j], bq), false, token);
        }
        carry_s = gmin(carry_s, ts);
        carry_p = gmax(carry_p, tp);
        if (k + 1 < nch) __syncthreads();
    }
    if (threadIdx.x == 0) st_guard<PACK>(&Gd.sylo[H], INFINITY, true, token);
}
__global__ void __launch_bounds__(kRowScanBlock) k_window_rowscan(WinGeom Q, WinGuard Gd) {
    __shared__ double red[2][kRowScanBlock / 64];
    row_guard_scan<kRowScanBlock, 1, false>(Q, Gd, red, 0);
}

// A row-guard value.  Packed (formed in the same launch, k_window_tile): the word is polled with
// sc1 loads until it carries this build's token; one that never does reads as `worst` (-inf for
// sylo, +inf for pyhi: every row a candidate row, so the windows only grow and stay complete).
// fp32 values rounded outward (sylo down, pyhi up) are sound bounds likewise.  Not packed: the
// double k_window_rowscan wrote (an earlier launch).
// `stalls` counts the words read at the spin limit (kWinStallWord, CBF_STAT_GUARD_STALLS).
__device__ __forceinline__ double ld_guard(const double* p, bool packed, int32_t token, double worst, int& stalls) {
    if (!packed) return *p;
    if (CBF_WIN_SPIN_LIMIT < 0) {  // (test build tests/_lib/libcbf_winnowait.so)
        ++stalls;
        return worst;
    }
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    for (long spins = 0;; ++spins) {
        const unsigned long long w = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int32_t)(w >> 32) == token) return (double)__uint_as_float((unsigned)w);
        if (spins >= CBF_WIN_SPIN_LIMIT) {
            ++stalls;
            return worst;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The rows of an ego at window row r, y: [r - Kd, r + Ku] (rows beyond are out of range).  The
// first kWinPre bounds each way are loaded together (sylo is non-decreasing and pyhi
// non-increasing away from r, so the test is monotone in k and Ku counts its failures); a window
// taller than that continues one row at a time.
constexpr int kWinPre = 4;
__device__ __forceinline__ void win_rows(const KP& P, const double* __restrict__ sylo,
                                         const double* __restrict__ pyhi, int r, int lo, int H, double y, int& Kd,
                                         int& Ku, bool packed, int32_t token, int& stalls) {
    double su[kWinPre], pd[kWinPre];
#pragma unroll
    for (int k = 0; k < kWinPre; ++k) {
        su[k] = r + k + 1 < H ? ld_guard(sylo + r + k + 1, packed, token, -INFINITY, stalls) : INFINITY;  // beyond: none
        pd[k] = r - k - 1 >= lo ? ld_guard(pyhi + r - k - 1, packed, token, INFINITY, stalls) : -INFINITY;
    }
    Ku = 0;
    Kd = 0;
#pragma unroll
    for (int k = 0; k < kWinPre; ++k) {
        Ku += !(su[k] - y > P.win_d) ? 1 : 0;
        Kd += !(y - pd[k] > P.win_d) ? 1 : 0;
    }
    if (Ku == kWinPre)
        while (r + Ku + 1 < H && !(ld_guard(sylo + r + Ku + 1, packed, token, -INFINITY, stalls) - y > P.win_d)) ++Ku;
    if (Kd == kWinPre)
        while (r - Kd - 1 >= lo && !(y - ld_guard(pyhi + r - Kd - 1, packed, token, INFINITY, stalls) > P.win_d)) ++Kd;
}

// 32-bit byte offsets into the lattice-ordered arrays (windows of < 2^28 agents, check_lattice)
__device__ __forceinline__ float2 ld_rsp(const float2* __restrict__ a, int t) {
    return *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(a) + ((uint32_t)t << 3));
}

// ---- the window filter: LDS tiles -----------------------------------
// A block is a tile of kTileR lattice rows x kTileW columns (one wave per tile row).  It stages
// the tile plus kTileKS halo rows and kTileKC halo columns of positions, nominal controls and
// column extents in LDS with coalesced loads (one round trip), then every candidate, sentinel and
// hit is read from LDS at a fixed offset from the ego's own slot: no per-lane gather chains.  Hits
// are bits of a register mask over the (7 rows x 5 columns) window, assembled from LDS after the
// scan.  An ego whose row window or column walk leaves the staged halo takes win_direct (global
// memory, unbounded), as in the untiled form.
constexpr int kTileW = 64;  // columns of a tile (one wave per tile row)
#ifndef CBF_TILE_R
#define CBF_TILE_R 8  // lattice rows (waves) per tile (4: 43.0 us, 8: 41.3 us per launch at 1 M agents)
#endif
constexpr int kTileR = CBF_TILE_R;
// (the launch's first block forms the row guard with a block scan over power-of-two waves: a tile of
// 6 or 7 rows left every guard word unformed, read at its spin limit -- exact, 0.78 s per launch)
static_assert(kTileR >= 2 && (kTileR & (kTileR - 1)) == 0, "tile rows: a power of two");
constexpr int kTileT = kTileR * 64;  // threads per tile block
constexpr int kTileKS = 3;  // rows each side (the row guard's window up to +-3)
constexpr int kTileKC = 3;  // columns each side (candidates to +-2, sentinels to +-3)
constexpr int kTileRows = kTileR + 2 * kTileKS, kTileCols = kTileW + 2 * kTileKC, kTileN = kTileRows * kTileCols;
constexpr int kTileGuard = kTileR + kWinPre - 1;  // sylo / pyhi values a tile needs
struct TileLds {
    double2 p[kTileN];
    double2 u[kTileN];
    float2 g[kTileN];  // column extents (fp32, outward) of the staged agents
    double sy[kTileGuard], py[kTileGuard];
};

// The unbounded form for one lane (rare): every row of [r - Kd, r + Ku] walked outward from the
// ego's column until its sentinels hold, hits assembled row by row (ego_add: the overflow path of
// the cell-list filter, same rows, same minima).  With f = 0 (FZ), candidates and sentinels inside
// the block's staged tile (rows tr0 .., columns tc0 .., kTileRows x kTileCols) are read from LDS,
// the rest from memory: the walk is one lane's chain of dependent reads, and from LDS it no longer holds
// its block into the launch's tail.  A staged sentinel is the fp32 column extent (a sorted row's:
// its own x rounded outward), at most one ulp looser than the exact x: a walk stops at the same
// column or one later, whose candidates then fail the cull test, so the hits are the same.
template <bool FZ>
__device__ __forceinline__ void win_direct(const KP& P, Ego& E, long w, int r, int c, int W, int Kd, int Ku,
                                        const double2* __restrict__ pos, const double2* __restrict__ u0,
                                        const float2* __restrict__ rsp, const int32_t* __restrict__ srt,
                                        double& smin, const double2* lp, const double2* lu, const float2* lg,
                                        int tr0, int tc0) {
    E.bq0 = E.bq1 = E.bq2 = E.bq3 = INFINITY;
    E.present = 0u;
    E.count = 0;
    smin = INFINITY;
    auto cand = [&](long j, bool st, int li) {
        const double2 p = st ? lp[li] : pos[j];
        const double e0 = p.x - E.r0, e1 = p.y - E.r1;
        const double s = e0 * e0 + e1 * e1;
        if (!(s < P.cull_t && s > 0)) return;
        smin = pmin(smin, s);
        const double2 v = st ? lu[li] : u0[j];
        ego_add<FZ>(P, E, p.x, p.y, v.x, v.y);
    };
    for (int dr = -Kd; dr <= Ku; ++dr) {
        const long b = w + (long)dr * W;
        // the row's sorted flag (a sorted row's column extents are its agents' own x); with FZ read
        // from memory only once the walk leaves the staged tile, so a walk inside it makes no memory
        // access (the general instantiation reads every sentinel from memory anyway)
        int so = FZ ? -1 : (srt[r + dr] != 0 ? 1 : 0);
        auto sorted_row = [&]() {
            if (so < 0) so = srt[r + dr] != 0 ? 1 : 0;
            return so != 0;
        };
        const int lr = r + dr - tr0, lb = lr * kTileCols - tc0;
        const bool srow = (unsigned)lr < (unsigned)kTileRows;
        // (f = 0 only: the general instantiation's walk has no registers to spare for it)
        auto staged = [&](int cc) { return FZ && srow && (unsigned)(cc - tc0) < (unsigned)kTileCols; };
        for (int dc = 0; c + dc < W; ++dc) {  // the column itself, then right
            const int cc = c + dc;
            cand(b + dc, staged(cc), lb + cc);
            if (cc + 1 >= W) break;
            const double sx = staged(cc + 1) ? (double)lg[lb + cc + 1].x
                                             : (sorted_row() ? pos[b + dc + 1].x : (double)rsp[b + dc + 1].x);
            if (sx - E.r0 > P.win_d) break;
        }
        for (int dc = -1; c + dc >= 0; --dc) {  // left
            const int cc = c + dc;
            cand(b + dc, staged(cc), lb + cc);
            if (cc - 1 < 0) break;
            const double sx = staged(cc - 1) ? (double)lg[lb + cc - 1].y
                                             : (sorted_row() ? pos[b + dc - 1].x : (double)rsp[b + dc - 1].y);
            if (E.r0 - sx > P.win_d) break;
        }
    }
}

template <bool FZ, bool ST, bool IN>
__global__ void __launch_bounds__(kTileT) __attribute__((amdgpu_waves_per_eu((IN || ST) ? 1 : CBF_TILE_WPE))) k_window_tile(KP P, WinBounds B, WinGeom Q, int er0, int tiles_x,
                                                        const double2* __restrict__ pos,
                                                        const double2* __restrict__ u0,
                                                        const float2* __restrict__ rsp, WinGuard Gd,
                                                        int32_t* __restrict__ sctl, double T,
                                                        double2* __restrict__ pos_out, double2* __restrict__ u,
                                                        int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                        unsigned long long* __restrict__ stats,
                                                        int32_t* __restrict__ hardq, HardRec* __restrict__ qrec,
                                                        long qcap) {
    __shared__ TileLds L;
    const double* __restrict__ sylo = Gd.sylo;
    const double* __restrict__ pyhi = Gd.pyhi;
    const int W = Q.W;
    const long nwin = (long)W * Q.rows;
    const int bx = xcd_block();
    // tile rows in the order last, 0, 1, ...: the window's two edge tile rows -- where a consensus
    // lattice's rows lose their x order and the rare walks (win_direct) happen -- run in the
    // launch's first round, so that no walk sits in its tail (speed only: any order is correct)
    const int tl = bx / tiles_x, tx = bx - tl * tiles_x;
    const int ty = tl == 0 ? (int)gridDim.x / tiles_x - 1 : tl - 1;
    const int r0 = er0 + ty * kTileR, c0 = tx * kTileW;  // window rows
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = r0 + wv, c = c0 + lane;
    const long w = (long)r * W + c;
    const bool inside = r < Q.rows && c < W;
    if (IN && ST && stats && (int)blockIdx.x == (int)gridDim.x - 1 && threadIdx.x < 64) stat_snapshot(stats);
    if (sctl[2] != 0) {  // the workspace is bound to another shape: report, touch nothing else
        lattice_error_tail(W, Q.row0 + B.own_lo / W, Q.row0 + B.own_hi / W, Q.row0, nwin, inside ? w : nwin, u,
                           status, cnt, stats, nullptr, 0, hardq);
        return;
    }
    // fold: the row guard without the k_window_rowscan launch.  The launch's first block
    // (dispatched first, so resident while any other block waits) forms sylo / pyhi from the
    // build's row extents and stores each value as one 64-bit word {fp32 value rounded outward,
    // the build's token} with an sc1 store; a reader polls the words it needs with sc1 loads until
    // they carry the token (ld_guard), so a block that starts after the guard is formed pays no
    // extra round trip and none waits on a done word.  (Where processes time-share the GPU the
    // first block can stall for long; cbf_params.launch_flags CBF_LAUNCH_SEPARATE_GUARD then
    // selects the separate scan kernel: fold = false.)  The build's choice, recorded in the
    // workspace header, decides (kWinModeWord).
    __shared__ double gred[2][kTileT / 64];
    const bool fold = sctl[kWinModeWord] != kGuardSeparate;
    const int32_t token = fold ? guard_token(sctl[kWinTokenWord]) : 0;  // written by the build (an earlier launch)
    if (fold && blockIdx.x == 0) row_guard_scan<kTileT, CBF_GUARD_PER, true>(Q, Gd, gred, token);
    // stage the tile with its halo (beyond the lattice: +-inf positions, which no test passes, and
    // column extents that exclude nothing beyond the row ends).  Every global load of the block --
    // each thread's (at most kStageK) entries: position, nominal control, the row's sorted flag and
    // the column extents, and the row-guard words' first poll -- is issued before any is waited
    // for: one memory round trip (a loop of dependent loads took four, a third of a block's life).
    // The extents are loaded for every row (the stale ones of a sorted row go unused).
    constexpr int kStageK = (kTileN + kTileT - 1) / kTileT;
    double2 sp[kStageK], su[kStageK];
    float2 sg[kStageK];
    int ss[kStageK];
    bool sv[kStageK];
#pragma unroll
    for (int k = 0; k < kStageK; ++k) {
        const int i = threadIdx.x + k * kTileT;
        const int lr = i / kTileCols, lc = i - lr * kTileCols;
        const int rr = r0 - kTileKS + lr, cc = c0 - kTileKC + lc;
        sv[k] = i < kTileN && rr >= Q.cr0 && rr < Q.cr1 && cc >= 0 && cc < W;
        // branch-free: an entry outside the window loads agent 0 (discarded below), so that no
        // load waits on another's condition
        const int t = sv[k] ? rr * W + cc : 0;
        sp[k] = ld_slot(pos, t);
        su[k] = ld_slot(u0, t);
        sg[k] = ld_rsp(rsp, t);
        ss[k] = Gd.srt[sv[k] ? rr : 0];
    }
    int stalls = 0;
    const int ga = r0 + 1 + (int)threadIdx.x, gb = r0 - kWinPre + (int)threadIdx.x;
    double gsy = INFINITY, gpy = -INFINITY;
    auto poll_guard = [&]() {
        if (threadIdx.x < kTileGuard) {
            if (ga < Q.cr1) gsy = ld_guard(sylo + ga, fold, token, -INFINITY, stalls);
            if (gb >= Q.cr0) gpy = ld_guard(pyhi + gb, fold, token, INFINITY, stalls);
        }
    };
    if (!CBF_TILE_EARLY_ROWS) poll_guard();
#pragma unroll
    for (int k = 0; k < kStageK; ++k) {
        const int i = threadIdx.x + k * kTileT;
        if (i >= kTileN) continue;
        if (sv[k]) {
            L.p[i] = sp[k];
            L.u[i] = su[k];
            // a sorted row's column extents are its agents' own x (outward to fp32); the build
            // stored extents for the other rows only
            L.g[i] = ss[k] ? make_float2(f32_down(sp[k].x), f32_up(sp[k].x)) : sg[k];
        } else {
            const int lc = i - (i / kTileCols) * kTileCols, cc = c0 - kTileKC + lc;
            const double v = cc < 0 ? -INFINITY : INFINITY;
            L.p[i] = make_double2(v, v);
            L.u[i] = make_double2(0.0, 0.0);
            L.g[i] = make_float2(INFINITY, -INFINITY);
        }
    }
    if (!CBF_TILE_EARLY_ROWS && threadIdx.x < kTileGuard) {
        L.sy[threadIdx.x] = gsy;
        L.py[threadIdx.x] = gpy;
    }
    __syncthreads();
    const bool act = inside && w >= B.own_lo && w < B.own_hi;
    const int e = (wv + kTileKS) * kTileCols + lane + kTileKC;  // the ego's slot in the tile
    Ego E;
    bool fin = false;
    if (act) {
        const double2 pe = L.p[e], ve = L.u[e];
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
        fin = isfinite(pe.x) && isfinite(pe.y);
    }
    unsigned long long hm = 0;  // hit bits (dr + 3) * 8 + (dc + 2): one byte per row
    double d2 = INFINITY;
    // FZ (f = 0) and CBF_TILE_FUSED_FLUSH: each hit's row_g goes into its quadrant minimum as the
    // candidate is tested (the coordinate differences reused: e = -d exactly up to the sign of a
    // zero, which neither |d0| + |d1| nor the d < 0 tests see); the minima are used where the
    // quadrant terms are finite (else the hits are taken row by row from hm, below)
    constexpr bool kFused = FZ && CBF_TILE_FUSED_FLUSH;
    double g0 = INFINITY, g1 = INFINITY, g2 = INFINITY, g3 = INFINITY;
    const unsigned long long kb = (unsigned long long)__double_as_longlong(P.k);
    const unsigned khi = (unsigned)(kb >> 32), knhi = khi ^ 0x80000000u, klo = (unsigned)kb;
    auto cand = [&](int off) -> unsigned {
        const double2 q = L.p[off];
        const double e0 = q.x - E.r0, e1 = q.y - E.r1;
        const double s = e0 * e0 + e1 * e1;
        const bool hit = s < P.cull_t && s > 0;
        if (ST && hit) d2 = pmin(d2, s);
        if (kFused && hit) {
            const double2 v = L.u[off];
            const bool nx = e0 > 0, ny = e1 > 0;  // d0 < 0, d1 < 0
            const double ksx = __hiloint2double((int)(nx ? knhi : khi), (int)klo);
            const double ksy = __hiloint2double((int)(ny ? knhi : khi), (int)klo);
            const double Hh = fma(ksy, E.r3 - v.y, fma(ksx, E.r2 - v.x, fabs(e0) + fabs(e1)));
            const double g = P.gamma * (Hh - P.dmin);
            if (!nx && !ny) g0 = vmin_f64(g0, g);
            if (nx && !ny) g1 = vmin_f64(g1, g);
            if (!nx && ny) g2 = vmin_f64(g2, g);
            if (nx && ny) g3 = vmin_f64(g3, g);
        }
        return hit ? 1u : 0u;
    };
    auto row_bits = [&](int dr) {  // the row's three hit bits (dc = -1, 0, 1 at bits 1, 2, 3 of its byte)
        const int b = e + dr * kTileCols;
        const unsigned rb = (cand(b - 1) << 1) | (dr != 0 ? cand(b) << 2 : 0u) | (cand(b + 1) << 3);  // (not itself)
        hm |= (unsigned long long)rb << ((dr + 3) * 8);
    };
    // CBF_TILE_EARLY_ROWS: rows -1, 0, +1 are tested before the row guard is read (so that a block
    // of the launch's first round does this work while the first block forms the guard).  Rows the
    // guard would have left out yield no hit: it proves their agents out of range, so hm, the
    // quadrant minima and d2 come out the same.
    // column-sentinel thresholds in fp32: a sentinel x with x > thR (x < thL) proves the columns
    // from it on out of range, since then x - r0 >= win_dn > win_d in real arithmetic and so in
    // fp64 (rounding is monotone); thR is r0 + win_dn rounded up (fp64, then to fp32 outward) and
    // thL likewise down.  At most one fp32 ulp looser than the fp64 test of the extents: a looser
    // bound only widens a window.  (Non-finite or huge coordinates give +-inf: every column needed.)
    float thR = INFINITY, thL = -INFINITY;
    if (fin) {
        const double tr = E.r0 + P.win_dn, tl = E.r0 - P.win_dn;
        thR = f32_up(tr + (fabs(tr) * 0x1p-50 + 0x1p-1070));
        thL = f32_down(tl - (fabs(tl) * 0x1p-50 + 0x1p-1070));
    }
    unsigned pR0 = 0, pL0 = 0;  // rows -1..+1 whose sentinel does not hold (EARLY_ROWS: masked below)
    if (CBF_TILE_EARLY_ROWS) {
        if (fin) {
#pragma unroll
            for (int dr = -1; dr <= 1; ++dr) {
                row_bits(dr);
                const int b = e + dr * kTileCols;
                if (!(L.g[b + 2].x > thR)) pR0 |= 1u << (dr + 3);
                if (!(L.g[b - 2].y < thL)) pL0 |= 1u << (dr + 3);
            }
        }
        poll_guard();
        if (threadIdx.x < kTileGuard) {
            L.sy[threadIdx.x] = gsy;
            L.py[threadIdx.x] = gpy;
        }
        __syncthreads();
    }
    int Kd = -1, Ku = -1;
    bool slow = false;
    if (fin) {
        Ku = 0;
        Kd = 0;
#pragma unroll
        for (int k = 0; k < kWinPre; ++k) {
            Ku += !(L.sy[wv + k] - E.r1 > P.win_d) ? 1 : 0;
            Kd += !(E.r1 - L.py[wv + kWinPre - 1 - k] > P.win_d) ? 1 : 0;
        }
        if (Ku > kTileKS || Kd > kTileKS) slow = true;  // beyond the staged rows: the unbounded form
    }
    // the wave's row range (DPP reductions; -1 for lanes without a window)
    const int KuW = (int)__ockl_wfred_max_u32((unsigned)(slow ? 0 : Ku + 1)) - 1;
    const int KdW = (int)__ockl_wfred_max_u32((unsigned)(slow ? 0 : Kd + 1)) - 1;
    unsigned pR = 0, pL = 0;  // rows (bit dr + 3) whose sentinel at c + 2 / c - 2 does not hold
    if (CBF_TILE_EARLY_ROWS && fin && !slow) {  // the early rows' sentinels, within the row window
        const unsigned win = ((2u << (Ku + 3)) - 1u) & ~((1u << (3 - Kd)) - 1u);  // bits -Kd .. Ku
        pR = pR0 & win;
        pL = pL0 & win;
    }
    for (int dr = -KdW; dr <= KuW; ++dr) {
        if (!(fin && !slow && dr >= -Kd && dr <= Ku)) continue;
        if (CBF_TILE_EARLY_ROWS && dr >= -1 && dr <= 1) continue;
        const int b = e + dr * kTileCols;
        row_bits(dr);
        if (!(L.g[b + 2].x > thR)) pR |= 1u << (dr + 3);
        if (!(L.g[b - 2].y < thL)) pL |= 1u << (dr + 3);
    }
    if (__ballot((pR | pL) != 0)) {  // columns c -+ 2 where a sentinel did not hold
        for (int dr = -KdW; dr <= KuW; ++dr) {
            const int b = e + dr * kTileCols, sh = (dr + 3) * 8;
            if ((pR >> (dr + 3)) & 1u) {
                hm |= (unsigned long long)(cand(b + 2) << 4) << sh;
                if (!(L.g[b + 3].x > thR)) slow = true;
            }
            if ((pL >> (dr + 3)) & 1u) {
                hm |= (unsigned long long)cand(b - 2) << sh;
                if (!(L.g[b - 3].y < thL)) slow = true;
            }
        }
    }
    const unsigned long long m_walk = __ballot(act && fin && slow);  // egos taking win_direct below
    EgoOut O;
    O.res = 0;
    O.w = -1;
    O.nbrs = 0;
    O.code = CBF_STATUS_IDLE;
    O.binding = false;
    O.seidel = false;
    O.viol = O.vorig = 0.0;
    O.d2 = INFINITY;
    if (act) {
        O.w = (int)w;
        const double q0 = quad_c(P, E, 0), q1 = quad_c(P, E, 1), q2 = quad_c(P, E, 2), q3 = quad_c(P, E, 3);
        const bool qfin = isfinite(q0) && isfinite(q1) && isfinite(q2) && isfinite(q3);
        if (fin && !slow) {
            // the hits from LDS: per-quadrant minima of row_g plus the quadrant terms, or row by row
            // (row_b) when a quadrant term is not finite -- the cell-list filter's two forms
            if (qfin) {
                E.count = __popcll(hm);
                // row_g<FZ> per hit (f = 0: its H with k's sign as a select of k's two high words --
                // -P.k flips exactly that bit -- instead of a multiply; same value bit for bit).  The
                // four quadrant minima are updated under the sign masks themselves (scalar mask logic,
                // no quadrant index), and a quadrant's presence is read off its minimum afterwards: a
                // present quadrant whose minimum stayed +inf (a NaN or +inf row) is a +inf plane,
                // which no solver step can violate or bind -- the same as an absent one.
                while (!kFused && hm) {
                    const int bit = __ffsll((long long)hm) - 1;
                    hm &= hm - 1;
                    const int off = e + ((bit >> 3) - 3) * kTileCols + (bit & 7) - 2;
                    const double2 q = L.p[off], v = L.u[off];
                    double g;
                    bool nx, ny;
                    if (FZ) {
                        const double d0 = E.r0 - q.x, d1 = E.r1 - q.y, d2 = E.r2 - v.x, d3 = E.r3 - v.y;
                        nx = d0 < 0;
                        ny = d1 < 0;
                        const double ksx = __hiloint2double((int)(nx ? knhi : khi), (int)klo);
                        const double ksy = __hiloint2double((int)(ny ? knhi : khi), (int)klo);
                        const double Hh = fma(ksy, d3, fma(ksx, d2, fabs(d0) + fabs(d1)));
                        g = P.gamma * (Hh - P.dmin);
                    } else {
                        int qd;
                        g = row_g<FZ>(P, E, q.x, q.y, v.x, v.y, qd);
                        nx = (qd & 1) != 0;
                        ny = (qd & 2) != 0;
                    }
                    // the hit's quadrant minimum, one v_min_f64 under that quadrant's lanes (exec-masked:
                    // the compare-and-select form took a compare and two selects per quadrant; the
                    // same value, see vmin_f64)
                    if (!nx && !ny) g0 = vmin_f64(g0, g);
                    if (nx && !ny) g1 = vmin_f64(g1, g);
                    if (!nx && ny) g2 = vmin_f64(g2, g);
                    if (nx && ny) g3 = vmin_f64(g3, g);
                }
                E.present = (g0 < INFINITY ? 1u : 0u) | (g1 < INFINITY ? 2u : 0u) | (g2 < INFINITY ? 4u : 0u) |
                            (g3 < INFINITY ? 8u : 0u);
                E.bq0 = g0 + q0;
                E.bq1 = g1 + q1;
                E.bq2 = g2 + q2;
                E.bq3 = g3 + q3;
            } else {  // a quadrant term is not finite: row by row (row_b), as the cell-list filter
                while (hm) {
                    const int bit = __ffsll((long long)hm) - 1;
                    hm &= hm - 1;
                    const int off = e + ((bit >> 3) - 3) * kTileCols + (bit & 7) - 2;
                    const double2 q = L.p[off], v = L.u[off];
                    ego_add<FZ>(P, E, q.x, q.y, v.x, v.y);
                }
            }
        } else if (fin) {  // the unbounded form, over the full row window (beyond the staged halo too)
            // a column walk (row window within the staged rows: the counts above are exact, since
            // fewer than kWinPre bounds failed) takes them as they are; a taller window reads the
            // row guard on from memory
            int kd = Kd, ku = Ku;
            if (Ku >= kWinPre || Kd >= kWinPre) win_rows(P, sylo, pyhi, r, Q.cr0, Q.cr1, E.r1, kd, ku, fold, token, stalls);
            win_direct<FZ>(P, E, w, r, c, W, kd, ku, pos, u0, rsp, Gd.srt, d2, L.p, L.u, L.g, r0 - kTileKS, c0 - kTileKC);
        }
        O.nbrs = E.count;
        if (ST) O.d2 = d2;
        ego_finish<FZ, ST, IN>(P, E, (int)w, (int)(w - B.own_lo), (int)w, T, pos_out, u, status, cnt, hardq,
                               bx % kSubQ, qrec, qcap, O);
    }
    // degradation counters (every instantiation; rare, so one wave-aggregated atomic each when
    // they occur): walks and guard words read at their spin limit, into the workspace header and,
    // with statistics, the CBF_STAT_WIN_WALKS / CBF_STAT_GUARD_STALLS words
    if (m_walk | __ballot(stalls > 0)) {
        int ns = stalls;
        for (int o = 32; o > 0; o >>= 1) ns += __shfl_xor(ns, o, 64);
        if (lane == 0) {
            const unsigned long long nw = (unsigned long long)__popcll(m_walk);
            unsigned long long* hdr = reinterpret_cast<unsigned long long*>(sctl);
            if (nw) atomicAdd(&hdr[kWinWalkWord / 2], nw);
            if (ns) atomicAdd(&hdr[kWinStallWord / 2], (unsigned long long)ns);
            if (ST && stats) {
                unsigned long long* sl = stats + 16 * stat_slot((long)bx * kTileR + wv);
                if (nw) atomicAdd(&sl[CBF_STAT_WIN_WALKS], nw);
                if (ns) atomicAdd(&sl[CBF_STAT_GUARD_STALLS], (unsigned long long)ns);
            }
        }
    }
    if (ST && stats) {
        const bool counted = O.res != 0 && O.w >= B.cnt_lo && O.w < B.cnt_hi;
        wave_stats(stats, (long)bx * kTileR + wv, counted && O.nbrs > 0, counted && O.seidel,
                   counted && O.res == 1, O.code, O.binding, O.viol, O.vorig, counted ? O.d2 : INFINITY);
    }
}

}  // namespace

namespace cbf {

// window-cull geometry a call can use: whole lattice (no halo), rows of 4 .. 2048 agents
bool window_cull_ok(int W, int rows, long n_ws, const CellWs& Wk) {
    return W >= 4 && W <= kWinMaxW && rows >= 1 && win_guard_bytes(rows) <= 16 * (size_t)n_ws && Wk.cs != nullptr;
}

bool window_fold(const cbf_params* p) { return !(p->launch_flags & CBF_LAUNCH_SEPARATE_GUARD); }

// the two degradation counters of a workspace's header (kWinWalkWord, kWinStallWord)
int window_counters(const void* workspace, size_t workspace_bytes, uint64_t* out, hipStream_t s) {
    if (!workspace || workspace_bytes < 256 || !out) return CBF_EINVAL;
    const uint64_t* hdr = reinterpret_cast<const uint64_t*>(workspace);
    if (hipError_t e = hipMemcpyAsync(out, hdr + kWinWalkWord / 2, 8, hipMemcpyDefault, s)) return (int)e;
    return (int)hipMemcpyAsync(out + 1, hdr + kWinStallWord / 2, 8, hipMemcpyDefault, s);
}

// threads of a build block for a window of the given rows: a window of few rows (one block per CU
// or fewer) takes 512-thread blocks, whose shorter per-thread chains end its latency-bound launch
// sooner (128 rows of 1,024 agents: 6.2 against 7.0 us; at 1,024 rows 256 threads are faster, 11.8
// against 13.9 us)
static int prep_threads(int rows) { return rows <= kPrepWideRows ? 2 * kPrepBlock : kPrepBlock; }

void window_prep(const CellWs& Wk, const WinGeom& Q, const double2* pos, double gain, double2* vel_out,
                 double2* copy_to, unsigned long long* ext_keys, int row_begin, int row_end, ExtSpec X,
                 bool fold, hipStream_t s) {
    const int nt = prep_threads(Q.cr1 - Q.cr0);
    const bool wide = nt != kPrepBlock;
    const auto prep = wide ? (Q.W <= 2 * nt ? k_window_prep<2, 2 * kPrepBlock> : k_window_prep<4, 2 * kPrepBlock>)
                           : (Q.W <= 2 * nt   ? k_window_prep<2, kPrepBlock>
                              : Q.W <= 4 * nt ? k_window_prep<4, kPrepBlock>
                                              : k_window_prep<8, kPrepBlock>);
    hipLaunchKernelGGL(prep, dim3(Q.cr1 - Q.cr0), dim3(nt), 24 * (size_t)Q.W, s, Q, pos, Wk.svel,
                       win_rsp(Wk), win_guard(Wk, Q.rows), gain, vel_out, copy_to, Wk.sctl, Wk.ncell, ext_keys,
                       row_begin, row_end, X, fold ? kGuardInFilter : kGuardSeparate);
    if (!fold)  // (else the filter's first block forms the row guard)
        hipLaunchKernelGGL(k_window_rowscan, dim3(1), dim3(kRowScanBlock), 0, s, Q, win_guard(Wk, Q.rows));
}

// The filter kernel of a window-cull advance of the egos of lattice rows [row_begin, row_end)
// (statistics over rows [cnt_begin, cnt_end)); pos_out (index (r - row_begin) W + c) must not
// overlap pos.  Where the row guard comes from is the build's choice (kWinModeWord), not p's.  The queued QPs are then solved by k_lattice_filter_hard (the caller launches it
// unless the solve is inline).
void window_filter(const cbf_params* p, const CellWs& Wk, const WinGeom& Q, int row_begin, int row_end,
                   int cnt_begin, int cnt_end, const double2* pos, double T, double2* pos_out, double2* u,
                   int32_t* status, int32_t* cnt, unsigned long long* stats, bool in, hipStream_t s,
                   hipEvent_t t_start, hipEvent_t t_stop) {
    const int W = Q.W;
    const long n = (long)W * Q.rows;
    const KP kp = make_kp(p);
    const WinBounds B = make_win_bounds(W, Q.row0, n, row_begin, row_end, cnt_begin, cnt_end, 0);
    const WinGuard Gd = win_guard(Wk, Q.rows);
    const int tiles_x = (W + kTileW - 1) / kTileW, tiles_y = (row_end - row_begin + kTileR - 1) / kTileR;
    const auto tile =
        in ? (stats ? (p->f_is_zero ? k_window_tile<true, true, true> : k_window_tile<false, true, true>)
                    : (p->f_is_zero ? k_window_tile<true, false, true> : k_window_tile<false, false, true>))
           : (stats ? (p->f_is_zero ? k_window_tile<true, true, false> : k_window_tile<false, true, false>)
                    : (p->f_is_zero ? k_window_tile<true, false, false> : k_window_tile<false, false, false>));
    if (t_start)  // the measurement hook: events carrying the launch's own start / end (hip_ext.h)
        hipExtLaunchKernelGGL(tile, dim3((unsigned)(tiles_x * tiles_y)), dim3(kTileT), 0, s, t_start, t_stop, 0u, kp, B,
                              Q, row_begin - Q.row0, tiles_x, pos, (const double2*)Wk.svel,
                              (const float2*)win_rsp(Wk), Gd, Wk.sctl, T, pos_out, u, status, cnt, stats, Wk.hardq,
                              Wk.qrec, Wk.qcap);
    else
        hipLaunchKernelGGL(tile, dim3((unsigned)(tiles_x * tiles_y)), dim3(kTileT), 0, s, kp, B, Q, row_begin - Q.row0,
                           tiles_x, pos, (const double2*)Wk.svel, (const float2*)win_rsp(Wk), Gd, Wk.sctl, T, pos_out,
                           u, status, cnt, stats, Wk.hardq, Wk.qrec, Wk.qcap);
}

}  // namespace cbf
