// swarm.hip -- nominal control, Euler, and the fused lattice-swarm timestep (gfx950).
//   graph-Laplacian consensus / cyclic pursuit   cross_and_rescue.py:108-125, meet_at_center.py:86-103
//   Euler                                        cross_and_rescue.py:173
//   whole timestep of a lattice swarm            SURVEY cfg3/cfg4 (cross_and_rescue.py:97-175 shape)
#include "cbf_device.hpp"
#include "cells.hpp"
#include "lattice.hpp"

using namespace cbf;

namespace {

inline int nblk(long n) { return (int)((n + kBlock - 1) / kBlock); }

constexpr int kExtSlotWords = 16;  // one 128-B line per extents slot (6 keys used)
#ifndef CBF_EXT_SLOTS
#define CBF_EXT_SLOTS 64
#endif
#ifndef CBF_EXT_WAVE
#define CBF_EXT_WAVE 0
#endif
constexpr int kExtSlots = CBF_EXT_SLOTS;  // slots per sub-step set (tools/ablate.py times the choices)
constexpr int kExtVals = 6;        // {ego min, ego max, owned max below guard, owned min above guard, owned min, max}
__host__ __device__ constexpr bool ext_is_min(int q) { return q == 0 || q == 3 || q == 4; }

struct ExtSpec {
    int own_begin, own_end, guard;
};

__global__ void __launch_bounds__(kBlock) k_consensus_csr(int n_dst, int self_offset, int n_group,
                                                          const double2* __restrict__ src,
                                                          const double2* __restrict__ anchors,
                                                          const int32_t* __restrict__ row_ptr,
                                                          const int32_t* __restrict__ col, int rotate, double rc,
                                                          double rs, double scale, double2* __restrict__ out) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= n_dst) return;
    const double2 xi = src[self_offset + k];
    double a0 = 0.0, a1 = 0.0;
    for (int t = row_ptr[k]; t < row_ptr[k + 1]; ++t) {
        const int j = col[t];
        const double2 xj = (j < n_group) ? src[j] : anchors[j - n_group];
        a0 = a0 + (xj.x - xi.x);
        a1 = a1 + (xj.y - xi.y);
    }
    double v0 = a0, v1 = a1;
    if (rotate) {  // (sum) @ [[rc, rs], [-rs, rc]] as OpenBLAS gemv evaluates it
        v0 = fma(a1, -rs, a0 * rc);
        v1 = fma(a1, rc, a0 * rs);
    }
    out[k] = make_double2(v0 * scale, v1 * scale);
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

__global__ void __launch_bounds__(kBlock) k_consensus_lattice(int W, int H, int row_begin, int row_end, int pos_row0,
                                                              const double2* __restrict__ pos, double scale,
                                                              double2* __restrict__ out) {
    const long k = (long)blockIdx.x * kBlock + threadIdx.x;
    const long nk = (long)(row_end - row_begin) * W;
    if (k >= nk) return;
    const int r = row_begin + (int)(k / W), c = (int)(k % W);
    const long w = (long)(r - pos_row0) * W + c;
    const double2 a = lattice_sum(pos, w, r, c, W, H);
    out[k] = make_double2(a.x * scale, a.y * scale);
}

__global__ void __launch_bounds__(kBlock) k_euler(int n, double2* __restrict__ pos, const double2* __restrict__ vel,
                                                  double T) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double2 p = pos[i], v = vel[i];
    pos[i] = make_double2(p.x + T * v.x, p.y + T * v.y);
}

// CBF_NOMINAL_IN_SCATTER: the Laplacian nominal control is computed by the scatter (K3) instead of
// K1, so it never makes an HBM round trip (tools/ablate.py, set nominal).
#ifndef CBF_NOMINAL_IN_SCATTER
#define CBF_NOMINAL_IN_SCATTER 1
#endif

// Lattice step K1, temporally coherent form: lanes walk the window agents in the previous step's
// cell order (identity on the first call), so consecutive lanes mostly share a cell; each run of
// equal cells in a wave takes its slots with ONE atomic (run length), and the later scatter
// writes nearly sequential slots.  Per-lane result bcs[t] = {cell, slot, agent} (12 B).
__global__ void __launch_bounds__(kBlock) k_lattice_nominal_bin_ordered(
    CellGrid G, int W, int H, int row_begin, int row_end, int win_row0, int win_rows, const double2* __restrict__ pos,
    double gain, double2* __restrict__ wvel, double2* __restrict__ vel_out, int32_t* __restrict__ count,
    const int32_t* __restrict__ order, const int32_t* __restrict__ start, long ncell, int3* __restrict__ bcs,
    int32_t* __restrict__ hardq, unsigned long long* __restrict__ ext_keys, ExtSpec X, int32_t* __restrict__ sctl) {
    const long t = (long)xcd_block() * kBlock + threadIdx.x;
    if (CBF_SCAN_EPOCH_BIN && t == 0) scan_epoch_advance(sctl);
    const long nwin = (long)win_rows * W;
    // hardq[2..4]: the previous build left a cell order for this window size and grid (else
    // identity); the order only permutes the work, so a stale one costs speed, never results
    const bool ordered = hardq[2] == 1 && hardq[3] == (int)nwin && hardq[4] == (int)ncell && hardq[5] == win_row0 &&
                         hardq[6] == H;
    int n_order = ordered ? start[ncell] : 0;
    n_order = n_order < 0 ? 0 : (n_order > nwin ? (int)nwin : n_order);
    if (t == 0) {  // hard-QP queue of this step's advance phase starts empty
        hardq[0] = 0;
        hardq[1] = 0;  // blocks of the queue kernel done (the last one empties the queue again)
    }
    int cell = -1;
    long w = -1;
    double2 p = make_double2(0.0, 0.0);
    if (t < nwin) {
        w = ordered ? (t < n_order ? order[t] : -1) : t;
        if (w >= 0 && w < nwin) {
            const int r = win_row0 + (int)(w / W);
            if ((r == 0 || r - 1 >= win_row0) && (r == H - 1 || r + 1 < win_row0 + win_rows)) {
                p = pos[w];
                cell = cell_coord(p.y, G.y0, G.inv_h, G.ny) * G.nx + cell_coord(p.x, G.x0, G.inv_h, G.nx);
            }
        }
    }
    const int lane = threadIdx.x & 63;
    if (ext_keys) {
        // y-extents of the INPUT positions for the halo guard of the sharded step (checked at the
        // next exchange): {min, max} over the computed rows [row_begin, row_end), and over the
        // owned rows {max y of rows < own_end - guard, min y of rows >= own_begin + guard, min,
        // max}.  Reduced per block, then one atomic per value into one of 64 slots on separate
        // 128-B lines (cross-XCD atomics on a shared line serialise at the memory side).
        __shared__ double red[6][kBlock / 64];
        double e[6] = {INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, -INFINITY};
        int any = 0;
        if (cell >= 0) {
            const int r = win_row0 + (int)(w / W);
            if (r >= row_begin && r < row_end) {
                e[0] = p.y;
                e[1] = p.y;
                any = 1;
            }
            if (r >= X.own_begin && r < X.own_end) {
                if (r < X.own_end - X.guard) e[2] = p.y;
                if (r >= X.own_begin + X.guard) e[3] = p.y;
                e[4] = p.y;
                e[5] = p.y;
                any = 1;
            }
        }
        // the common wave has one membership pattern for all its agents: two reductions (min and
        // max of y) instead of six
        const unsigned code = any ? ((e[0] != INFINITY ? 1u : 0u) | (e[2] != -INFINITY ? 2u : 0u) |
                                     (e[3] != INFINITY ? 4u : 0u) | (e[4] != INFINITY ? 8u : 0u))
                                  : 0u;
        const unsigned long long act = __ballot(any);
        const unsigned c0 = (unsigned)__shfl((int)code, act ? __ffsll((long long)act) - 1 : 0, 64);
        if (__ballot(any && code != c0) == 0) {
            const double mn = wave_min(any ? p.y : INFINITY), mx = wave_max(any ? p.y : -INFINITY);
            const bool has = act != 0;
            e[0] = (has && (c0 & 1u)) ? mn : INFINITY;
            e[1] = (has && (c0 & 1u)) ? mx : -INFINITY;
            e[2] = (has && (c0 & 2u)) ? mx : -INFINITY;
            e[3] = (has && (c0 & 4u)) ? mn : INFINITY;
            e[4] = (has && (c0 & 8u)) ? mn : INFINITY;
            e[5] = (has && (c0 & 8u)) ? mx : -INFINITY;
        } else {
#pragma unroll
            for (int q = 0; q < 6; ++q) e[q] = ext_is_min(q) ? wave_min(e[q]) : wave_max(e[q]);
        }
#if CBF_EXT_WAVE
        // per wave: lane 0 of every wave with an agent in range does the atomics (no block barrier)
        if (__ballot(any) && lane == 0) {
            unsigned long long* k = ext_keys + kExtSlotWords * ((t >> 6) & (kExtSlots - 1));
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (ext_is_min(q)) atomicMin(&k[q], dkey(e[q]));
                else atomicMax(&k[q], dkey(e[q]));
            }
        }
#else
        const int wid = threadIdx.x >> 6;
        if (lane == 0)
#pragma unroll
            for (int q = 0; q < 6; ++q) red[q][wid] = e[q];
        if (__syncthreads_or(any) && threadIdx.x == 0) {
            for (int v = 1; v < kBlock / 64; ++v)
#pragma unroll
                for (int q = 0; q < 6; ++q)
                    e[q] = ext_is_min(q) ? pmin(e[q], red[q][v]) : pmax(e[q], red[q][v]);
            unsigned long long* k = ext_keys + kExtSlotWords * (blockIdx.x & (kExtSlots - 1));
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (ext_is_min(q)) atomicMin(&k[q], dkey(e[q]));
                else atomicMax(&k[q], dkey(e[q]));
            }
        }
#endif
    }
    // runs of equal cells inside the wave: one atomic per run
    int cprev = __shfl_up(cell, 1, 64);
    const bool leader = lane == 0 || cell != cprev;
    const unsigned long long lm = __ballot(leader);
    const unsigned long long upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const int my_leader = 63 - __clzll(lm & upto);
    const unsigned long long above = lm & ~upto;
    const int next = above ? __ffsll((long long)above) - 1 : 64;
    int base = 0;
    if (leader && cell >= 0) base = atomicAdd(&count[cell], next - lane);
    base = __shfl(base, my_leader, 64);
    if (t >= nwin) return;
    if (cell < 0) {
        bcs[t] = make_int3(-1, 0, (int)w);
        return;
    }
#if !CBF_NOMINAL_IN_SCATTER
    const int r = win_row0 + (int)(w / W), c = (int)(w % W);
    const double2 a = lattice_sum(pos, w, r, c, W, H);
    const double2 u0 = make_double2(a.x * gain, a.y * gain);
    wvel[w] = u0;
    if (vel_out != wvel && r >= row_begin && r < row_end) vel_out[(long)(r - row_begin) * W + c] = u0;
#endif
    bcs[t] = make_int3(cell, base + lane - my_leader, (int)w);
}

__global__ void __launch_bounds__(kBlock) k_lattice_scatter_ordered(long nwin, const int3* __restrict__ bcs,
                                                                    const int32_t* __restrict__ start,
                                                                    const double2* __restrict__ pos,
                                                                    const double2* __restrict__ wvel,
                                                                    double2* __restrict__ spos,
                                                                    double2* __restrict__ svel,
                                                                    int32_t* __restrict__ sidx,
                                                                    float2* __restrict__ spos32,
                                                                    int32_t* __restrict__ order_state, long n,
                                                                    long ncell, int win_row0, int H, int W,
                                                                    int row_begin, int row_end, double gain,
                                                                    double2* __restrict__ vel_out) {
    const long t = (long)xcd_block() * kBlock + threadIdx.x;
    if (t == 0) {  // the cell order now exists for this window and grid: the next build walks it
        order_state[0] = 1;
        order_state[1] = (int)n;
        order_state[2] = (int)ncell;
        order_state[3] = win_row0;
        order_state[4] = H;
    }
    if (t >= nwin) return;
    const int3 b = bcs[t];
    if (b.x < 0) return;
    const int d = start[b.x] + b.y;
    const double2 p = pos[b.z];
    spos[d] = p;
#if CBF_NOMINAL_IN_SCATTER
    // K1's nominal control computed here: the agent's position is loaded anyway and its 4
    // lattice neighbours are mostly in L2 (cell order ~ lattice order), so the u0 round trip
    // through HBM (written by K1, gathered back here) disappears
    const int r = win_row0 + b.z / W, c = b.z % W;
    const double2 a = lattice_sum(pos, b.z, r, c, W, H);
    const double2 u0 = make_double2(a.x * gain, a.y * gain);
    svel[d] = u0;
    if (r >= row_begin && r < row_end) vel_out[(long)(r - row_begin) * W + c] = u0;
    (void)wvel;
#else
    svel[d] = wvel[b.z];
    (void)W, (void)row_begin, (void)row_end, (void)gain, (void)vel_out;
#endif
    sidx[d] = b.z;
#if CBF_SCAN32
    spos32[d] = make_float2((float)p.x, (float)p.y);
#endif
}


// Tail of the lattice filter for one owned ego whose QP rows are accumulated in E: solve at the
// origin or queue to the hard kernel, clip, Euler, outputs.  Returns 1 (done, *ny = new y) or 2.
// CBF_HARD_INLINE (off): a QP the origin does not solve is solved in place by solve_ego_lds (rolled
// loops, right-hand sides in the lane's LDS column `bl`, ~30 VGPRs) instead of being queued for
// k_lattice_filter_hard, which then is not launched (its launch + queue round trip was ~10 us a
// step for ~0.3 % of the egos).
#ifndef CBF_NT_STORES
#define CBF_NT_STORES 0
#endif
#ifndef CBF_HARD_INLINE
#define CBF_HARD_INLINE 0  // measured slower: advance 55.7 vs 51.9 us (tools/ablate.py, set hardinline)
#endif
template <bool FZ>
__device__ __forceinline__ int ego_finish(const KP& P, Ego& E, int W, int row_begin, int r, int c, double T,
                                          double2* __restrict__ pos_out, double2* __restrict__ u,
                                          int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                          int32_t* __restrict__ hardq, double* ny, int* bl = nullptr) {
    const double2 pe = make_double2(E.r0, E.r1);
    const long k = (long)(r - row_begin) * W + c;
    double ux, uy;
    int32_t st;
    if (E.count == 0) {
        ux = E.u0x;
        uy = E.u0y;
        st = CBF_STATUS_IDLE;
    } else {
        Sol S;
#if CBF_ABLATE >= 1
        S.x0 = S.x1 = 0.0;
        S.status = CBF_STATUS_OPTIMAL;
        S.iters = 0;
        S.viol = E.bq0 + E.bq1 + E.bq2 + E.bq3;
        asm volatile("" ::"v"(S.viol));
#else
        if (solve_easy(P, E, S)) {
        } else if (CBF_HARD_INLINE && bl) {
            S = solve_ego_lds(P, E, LaneCol{bl});
        } else {
            HardRec* q = reinterpret_cast<HardRec*>(hardq + kHardHeader);
            HardRec& h = q[atomicAdd(&hardq[0], 1)];
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
            h.k = (int)k;
            h.row = r;
            return 2;
        }
#endif
        clip_u(P, S, E, ux, uy);
        st = pack_status(S);
    }
    const double2 pn = make_double2(pe.x + T * ux, pe.y + T * uy);
#if CBF_NT_STORES
    // outputs are not read again by this kernel: non-temporal stores keep them from displacing
    // the cell-sorted candidate lines in L2
    __builtin_nontemporal_store(pn.x, &pos_out[k].x);
    __builtin_nontemporal_store(pn.y, &pos_out[k].y);
    __builtin_nontemporal_store(ux, &u[k].x);
    __builtin_nontemporal_store(uy, &u[k].y);
    __builtin_nontemporal_store(st, &status[k]);
    if (cnt) __builtin_nontemporal_store(E.count, &cnt[k]);
#else
    pos_out[k] = pn;
    u[k] = make_double2(ux, uy);
    status[k] = st;
    if (cnt) cnt[k] = E.count;
#endif
    *ny = pn.y;
    return 1;
}

// Lattice step K4: filter + clip + Euler for one owned agent at cell-sorted slot `slot`.
// QPs that the origin does not solve (after the strip pre-relaxation) are not solved here but
// appended, with their assembled state, to the hard queue: one such lane would otherwise make
// its whole wave run the Seidel path (and hold the registers for it); K5 solves them.
// Returns 0 (not an owned agent), 1 (done: outputs written, *ny = new y), 2 (queued).
template <bool FZ>
__device__ __forceinline__ int lattice_ego(const KP& P, const CellGrid& G, int W, int row_begin, int row_end,
                                           int win_row0, int slot, const double2* __restrict__ spos,
                                           const double2* __restrict__ svel, const int32_t* __restrict__ sidx,
                                           const int32_t* __restrict__ start, double T, double2* __restrict__ pos_out,
                                           double2* __restrict__ u, int32_t* __restrict__ status,
                                           int32_t* __restrict__ cnt, int32_t* __restrict__ hardq, int* hit_lds,
                                           const float2* __restrict__ spos32, double* ny, int* row, int* nbrs) {
    const int w = sidx[slot];
    const int r = win_row0 + w / W;
    const int c = w % W;
    *row = r;
    if (!(r >= row_begin && r < row_end)) return 0;
    const double2 pe = spos[slot], ve = svel[slot];
    Ego E;
    ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    const int cx = cell_coord(pe.x, G.x0, G.inv_h, G.nx);
    const int cy = cell_coord(pe.y, G.y0, G.inv_h, G.ny);
    const int xa = cx > 0 ? cx - 1 : 0;
    const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
    // pass 1: cheap cull test over the 3x3 cells, hits compacted into a per-lane LDS list;
    // pass 2: row assembly only for hits (keeps divergent lanes from paying assembly for
    // every candidate iteration of the wave)
    int rt0[3], rt1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int yy = cy + k - 1;
        const bool in = yy >= 0 && yy < G.ny;
        rt0[k] = in ? start[yy * G.nx + xa] : 0;
        rt1[k] = in ? start[yy * G.nx + xb + 1] : 0;
    }
#if CBF_SCAN_INLINE && CBF_SCAN_U > 0 && CBF_ABLATE == 0
    scan_rows_inline<FZ>(rt0, rt1, P, E, spos, svel);
    (void)hit_lds;
    (void)spos32;
#elif CBF_HIT_MASK && CBF_SCAN_U > 0 && CBF_ABLATE == 0
    {
        HitMask Hm;
        if (scan_rows_joint_mask(rt0, rt1, P, E, Hm, spos)) {
            flush_mask<FZ>(Hm, rt0, P, E, spos, svel);
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) scan_range_direct<FZ>(rt0[k], rt1[k], P, E, spos, svel);
        }
        (void)hit_lds;
        (void)spos32;
    }
#elif CBF_ABLATE < 3
    HitList Hl;
#if CBF_SCAN32
    // screen bound from the ego's own magnitude: a true neighbour lies within r of it
    const float t32 = screen_threshold(P.cull_t, pmax(fabs(E.r0), fabs(E.r1)) + sqrt(P.cull_t));
    constexpr bool kExact = true;
    if (t32 > 0.0f)
        scan_rows_joint32(rt0, rt1, t32, (float)E.r0, (float)E.r1, Hl, hit_lds, spos32);
    else
        Hl.n = kHitCap + 1;  // screen off (non-finite or huge coordinates): the exact direct scan
#elif CBF_SCAN_U > 0
    constexpr bool kExact = false;
    scan_rows_joint(rt0, rt1, P, E, Hl, hit_lds, spos);
#else
    constexpr bool kExact = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) scan_range(rt0[k], rt1[k], P, E, Hl, hit_lds, spos);
#endif
#if CBF_ABLATE < 2
    if (!Hl.overflowed()) {
#if CBF_BQ_LDS
        double* bq = reinterpret_cast<double*>(hit_lds + (kHitCap + 1) * kBlock);
#pragma unroll
        for (int q = 0; q < 4; ++q) bq[q * kBlock + threadIdx.x] = INFINITY;
        Hl.template flush_bq<FZ, kExact>(hit_lds, bq, P, E, spos, svel);
        E.bq0 = bq[threadIdx.x];
        E.bq1 = bq[kBlock + threadIdx.x];
        E.bq2 = bq[2 * kBlock + threadIdx.x];
        E.bq3 = bq[3 * kBlock + threadIdx.x];
#else
        Hl.template flush<FZ, kExact>(hit_lds, P, E, spos, svel);
#endif
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) scan_range_direct<FZ>(rt0[k], rt1[k], P, E, spos, svel);
    }
#else
    E.count = Hl.n;
    asm volatile("" ::"v"(E.count));
#endif
#endif
    *nbrs = E.count;
    // the lane's LDS column (its hit slots) is free again after the flush: the 8 right-hand sides
    // of an in-place solve (other lanes' columns may still be in use by their waves)
    int* bl = CBF_HIT_MASK ? nullptr : hit_lds + threadIdx.x;
    return ego_finish<FZ>(P, E, W, row_begin, r, c, T, pos_out, u, status, cnt, hardq, ny, bl);
}

// K4: one lane per cell-sorted slot; easy QPs solved in place, hard ones queued.
#ifndef CBF_FILTER_WPE
#define CBF_FILTER_WPE 0
#endif
#if CBF_FILTER_WPE > 0
#define CBF_FILTER_BOUNDS __launch_bounds__(kBlock, CBF_FILTER_WPE)
#else
#define CBF_FILTER_BOUNDS __launch_bounds__(kBlock)
#endif
template <bool FZ>
__global__ void CBF_FILTER_BOUNDS k_lattice_filter(KP P, CellGrid G, int W, int row_begin, int row_end,
                                                           int win_row0, long ncell, const double2* __restrict__ spos,
                                                           const double2* __restrict__ svel,
                                                           const int32_t* __restrict__ sidx,
                                                           const int32_t* __restrict__ start, double T,
                                                           double2* __restrict__ pos_out, double2* __restrict__ u,
                                                           int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                           int guard_rows, double* __restrict__ ext_part,
                                                           unsigned long long* __restrict__ solves,
                                                           int32_t* __restrict__ hardq,
                                                           const float2* __restrict__ spos32, int cnt_begin,
                                                           int cnt_end) {
    // hit rows + a dummy row (branch-free push) + 4 x fp64 per-quadrant minima (CBF_BQ_LDS)
    // (>= 16 ints per lane: also the lane's 8 fp64 right-hand sides of an in-place hard solve)
    static_assert(CBF_HIT_MASK || (kHitCap + 1) + (CBF_BQ_LDS ? 8 : 0) >= 16, "hit LDS too small for solve_ego_lds");
    __shared__ int hit_lds[CBF_HIT_MASK ? 1 : (kHitCap + 1) * kBlock + (CBF_BQ_LDS ? 8 * kBlock : 0)];
    const int bx = xcd_block();
    const int slot = bx * kBlock + threadIdx.x;
    const int total = start[ncell];
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    bool solved = false;
    if (slot < total) {
        double ny;
        int r, nb = 0;
        const int res = lattice_ego<FZ>(P, G, W, row_begin, row_end, win_row0, slot, spos, svel, sidx, start,
                                               T, pos_out, u, status, cnt, hardq, hit_lds, spos32, &ny, &r, &nb);
        solved = res != 0 && nb > 0 && r >= cnt_begin && r < cnt_end;
        if (res == 1) ext_accumulate(r, row_begin, row_end, guard_rows, ny, e0, e1, e2, e3);
    }
    if (solves) {  // wave-aggregated, spread over 64 counters on separate 128-B lines
        const unsigned long long m = __ballot(solved);
        if ((threadIdx.x & 63) == 0 && m)
            atomicAdd(&solves[16 * ((bx * (kBlock / 64) + (threadIdx.x >> 6)) & 63)],
                      (unsigned long long)__popcll(m));
    }
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, (long)bx * (kBlock / 64) + (threadIdx.x >> 6));
}

// K4, LDS-staged form (CBF_LDS_STAGE): the egos of a wave are consecutive cell-sorted slots, so
// the union of their three cell-row candidate ranges is three short contiguous slot segments
// (~210 agents at the cfg4 density).  The wave loads that union once, coalesced, into its own
// LDS region (positions and nominal controls), then every lane culls and assembles its own ~17
// candidates from LDS: no per-lane gathers, no hit list, no flush.  A wave whose union exceeds
// kStageCap (a sparse or wrapped region) takes the direct path from global memory.  Same rows,
// same per-quadrant minima as k_lattice_filter (the minimum is order-independent).
#ifndef CBF_LDS_STAGE
#define CBF_LDS_STAGE 0
#endif
constexpr int kStageCap = 256;

template <bool FZ>
__global__ void __launch_bounds__(kBlock) k_lattice_filter_lds(KP P, CellGrid G, int W, int row_begin, int row_end,
                                                               int win_row0, long ncell,
                                                               const double2* __restrict__ spos,
                                                               const double2* __restrict__ svel,
                                                               const int32_t* __restrict__ sidx,
                                                               const int32_t* __restrict__ start, double T,
                                                               double2* __restrict__ pos_out, double2* __restrict__ u,
                                                               int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                               unsigned long long* __restrict__ solves,
                                                               int32_t* __restrict__ hardq, int cnt_begin,
                                                               int cnt_end) {
    __shared__ double2 st_pos[kBlock / 64][kStageCap];
    __shared__ double2 st_vel[kBlock / 64][kStageCap];
    const int bx = xcd_block();
    const int slot = bx * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int total = start[ncell];
    bool act = false;
    int r = 0, c = 0;
    Ego E;
    int rt0[3] = {0, 0, 0}, rt1[3] = {0, 0, 0};
    if (slot < total) {
        const int w = sidx[slot];
        r = win_row0 + w / W;
        c = w % W;
        if (r >= row_begin && r < row_end) {
            act = true;
            const double2 pe = spos[slot], ve = svel[slot];
            ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
            const int cx = cell_coord(pe.x, G.x0, G.inv_h, G.nx);
            const int cy = cell_coord(pe.y, G.y0, G.inv_h, G.ny);
            const int xa = cx > 0 ? cx - 1 : 0;
            const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int yy = cy + k - 1;
                if (yy >= 0 && yy < G.ny) {
                    rt0[k] = start[yy * G.nx + xa];
                    rt1[k] = start[yy * G.nx + xb + 1];
                }
            }
        }
    }
    // wave union of the three row ranges
    int lo[3], len[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool ne = act && rt1[k] > rt0[k];
        int a = ne ? rt0[k] : 0x7FFFFFFF, b = ne ? rt1[k] : -1;
        for (int o = 32; o > 0; o >>= 1) {
            const int a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64);
            a = a2 < a ? a2 : a;
            b = b2 > b ? b2 : b;
        }
        lo[k] = a;
        len[k] = b > a ? b - a : 0;
    }
    const int off1 = len[0], off2 = len[0] + len[1], L = off2 + len[2];
    if (L <= kStageCap) {
#pragma unroll
        for (int j = 0; j < kStageCap / 64; ++j) {
            const int i = lane + 64 * j;
            if (i < L) {
                const int g = i >= off2 ? lo[2] + (i - off2) : (i >= off1 ? lo[1] + (i - off1) : lo[0] + i);
                st_pos[wid][i] = spos[g];
                st_vel[wid][i] = svel[g];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (act) {
#if CBF_LDS_STAGE == 2
            // pass 1: cull test only, hits as a bit mask per row range; pass 2: assembly per hit
            // (the wave iterates max-hits times instead of max-candidates times)
            unsigned m[3] = {0u, 0u, 0u};
            bool wide = false;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int base = (k == 0 ? 0 : (k == 1 ? off1 : off2)) - lo[k];
                wide = wide || rt1[k] - rt0[k] > 32;
                const int te = rt1[k] - rt0[k] > 32 ? rt0[k] + 32 : rt1[k];
                for (int t = rt0[k]; t < te; ++t) {
                    const double2 pj = st_pos[wid][base + t];
                    const double e0 = pj.x - E.r0, e1 = pj.y - E.r1;
                    const double s = e0 * e0 + e1 * e1;
                    if (s < P.cull_t && s > 0) m[k] |= 1u << (t - rt0[k]);
                }
            }
            if (!wide) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int base = (k == 0 ? 0 : (k == 1 ? off1 : off2)) - lo[k] + rt0[k];
                    while (m[k]) {
                        const int b = __ffs((int)m[k]) - 1;
                        m[k] &= m[k] - 1u;
                        const double2 pj = st_pos[wid][base + b];
                        const double2 vj = st_vel[wid][base + b];
                        ego_add<FZ>(P, E, pj.x, pj.y, vj.x, vj.y);
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) scan_range_direct<FZ>(rt0[k], rt1[k], P, E, spos, svel);
            }
#else
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int base = (k == 0 ? 0 : (k == 1 ? off1 : off2)) - lo[k];
                for (int t = rt0[k]; t < rt1[k]; ++t) {
                    const double2 pj = st_pos[wid][base + t];
                    const double e0 = pj.x - E.r0, e1 = pj.y - E.r1;
                    const double s = e0 * e0 + e1 * e1;
                    if (!(s < P.cull_t && s > 0)) continue;
                    const double2 vj = st_vel[wid][base + t];
                    ego_add<FZ>(P, E, pj.x, pj.y, vj.x, vj.y);
                }
            }
#endif
        }
    } else if (act) {
#pragma unroll
        for (int k = 0; k < 3; ++k) scan_range_direct<FZ>(rt0[k], rt1[k], P, E, spos, svel);
    }
    bool solved = false;
    if (act) {
        double ny;
        const int res = ego_finish<FZ>(P, E, W, row_begin, r, c, T, pos_out, u, status, cnt, hardq, &ny);
        solved = res != 0 && E.count > 0 && r >= cnt_begin && r < cnt_end;
    }
    if (solves) {
        const unsigned long long m = __ballot(solved);
        if (lane == 0 && m)
            atomicAdd(&solves[16 * ((bx * (kBlock / 64) + wid) & 63)], (unsigned long long)__popcll(m));
    }
}

// K5: the queued hard QPs (state assembled by K4), 64-lane blocks spread over the CUs.
__global__ void __launch_bounds__(64) k_lattice_filter_hard(KP P, int row_begin, int row_end, double T,
                                                            double2* __restrict__ pos_out, double2* __restrict__ u,
                                                            int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                            int guard_rows, double* __restrict__ ext_part,
                                                            int32_t* __restrict__ hardq, int cap) {
    (void)cap;
    const int nq = hardq[0];
    const HardRec* q = reinterpret_cast<const HardRec*>(hardq + kHardHeader);
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    for (int i = blockIdx.x * 64 + threadIdx.x; i < nq; i += gridDim.x * 64) {
        const HardRec& h = q[i];
        Ego E;
        E.r0 = h.r0;
        E.r1 = h.r1;
        E.r2 = h.r2;
        E.r3 = h.r3;
        E.u0x = h.u0x;
        E.u0y = h.u0y;
        E.bq0 = h.bq0;
        E.bq1 = h.bq1;
        E.bq2 = h.bq2;
        E.bq3 = h.bq3;
        E.present = (unsigned)h.present;
        E.count = h.count;
        const Sol S = solve_ego(P, E);
        double ux, uy;
        clip_u(P, S, E, ux, uy);
        const double2 pn = make_double2(E.r0 + T * ux, E.r1 + T * uy);
        pos_out[h.k] = pn;
        u[h.k] = make_double2(ux, uy);
        status[h.k] = pack_status(S);
        if (cnt) cnt[h.k] = E.count;
        ext_accumulate(h.row, row_begin, row_end, guard_rows, pn.y, e0, e1, e2, e3);
    }
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, blockIdx.x);
    hard_queue_done(hardq);
}


constexpr int kFinBlock = 1024;
__global__ void __launch_bounds__(kFinBlock) k_extents_finalize(int nparts, const double* __restrict__ part,
                                                                double* __restrict__ out) {
    double a = INFINITY, b = -INFINITY, c = -INFINITY, d = INFINITY;
    // 8 records in flight per thread (the reduction is latency-bound on one block)
    for (int i0 = threadIdx.x; i0 < nparts; i0 += 8 * kFinBlock) {
        double4 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * kFinBlock;
            r[k] = i < nparts ? reinterpret_cast<const double4*>(part)[i]
                              : make_double4(INFINITY, -INFINITY, -INFINITY, INFINITY);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a = pmin(a, r[k].x);
            b = pmax(b, r[k].y);
            c = pmax(c, r[k].z);
            d = pmin(d, r[k].w);
        }
    }
    a = wave_min(a);
    b = wave_max(b);
    c = wave_max(c);
    d = wave_min(d);
    __shared__ double red[4][kFinBlock / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wid] = a;
        red[1][wid] = b;
        red[2][wid] = c;
        red[3][wid] = d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < kFinBlock / 64; ++q) {
            red[0][0] = pmin(red[0][0], red[0][q]);
            red[1][0] = pmax(red[1][0], red[1][q]);
            red[2][0] = pmax(red[2][0], red[2][q]);
            red[3][0] = pmin(red[3][0], red[3][q]);
        }
        out[0] = red[0][0];
        out[1] = red[1][0];
        out[2] = red[2][0];
        out[3] = red[3][0];
    }
}

__global__ void k_halo_guard(const double* __restrict__ E, long stride, int ws, int rank, double radius,
                             int32_t* __restrict__ flag) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const double rm = radius * (1.0 + 1e-9) + 1e-12;
    const double* me = E + (long)rank * stride;
    const double ymin = me[0], ymax = me[1];
    int bad = 0;
    for (int q = 0; q < ws; ++q) {
        const double* o = E + (long)q * stride;
        if (q < rank) {  // rows below: rank-1's rows outside our halo, everything of lower ranks
            const double lim = (q == rank - 1) ? o[2] : o[1];
            if (!(ymin - lim > rm)) bad = 1;
        } else if (q > rank) {
            const double lim = (q == rank + 1) ? o[3] : o[0];
            if (!(lim - ymax > rm)) bad = 1;
        }
    }
    if (bad) flag[0] |= 1;
}

}  // namespace

namespace cbf {
void launch_extents_finalize(int nparts, const double* part, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_extents_finalize, dim3(1), dim3(kFinBlock), 0, s, nparts, part, out);
}
}  // namespace cbf

extern "C" int cbf_halo_guard(const double* ext_all, int64_t stride, int32_t world_size, int32_t rank, double radius,
                              int32_t* flag, void* stream) {
    if (!ext_all || !flag || world_size < 1 || rank < 0 || rank >= world_size || stride < 4) return CBF_EINVAL;
    hipLaunchKernelGGL(k_halo_guard, dim3(1), dim3(64), 0, (hipStream_t)stream, ext_all, (long)stride, world_size,
                       rank, radius, flag);
    return (int)hipGetLastError();
}

extern "C" int cbf_consensus_csr(int32_t n_dst, int32_t self_offset, int32_t n_group, const double* src,
                                 const double* anchors, const int32_t* row_ptr, const int32_t* col, int32_t rotate,
                                 double rc, double rs, double scale, double* out, void* stream) {
    if (n_dst < 0 || self_offset < 0 || n_group < 0 || self_offset + n_dst > n_group) return CBF_EINVAL;
    if (n_dst == 0) return 0;
    if (!src || !row_ptr || !out) return CBF_EINVAL;
    hipLaunchKernelGGL(k_consensus_csr, dim3(nblk(n_dst)), dim3(kBlock), 0, (hipStream_t)stream, n_dst, self_offset,
                       n_group, reinterpret_cast<const double2*>(src), reinterpret_cast<const double2*>(anchors),
                       row_ptr, col, rotate, rc, rs, scale, reinterpret_cast<double2*>(out));
    return (int)hipGetLastError();
}

extern "C" int cbf_consensus_lattice(int32_t W, int32_t H, int32_t row_begin, int32_t row_end, int32_t pos_row0,
                                     const double* pos, double scale, double* out, void* stream) {
    if (W <= 0 || H <= 0 || row_begin < 0 || row_end > H || row_begin > row_end) return CBF_EINVAL;
    if (pos_row0 > (row_begin > 0 ? row_begin - 1 : 0)) return CBF_EINVAL;
    if (row_end == row_begin) return 0;
    if (!pos || !out) return CBF_EINVAL;
    const long nk = (long)(row_end - row_begin) * W;
    hipLaunchKernelGGL(k_consensus_lattice, dim3(nblk(nk)), dim3(kBlock), 0, (hipStream_t)stream, W, H, row_begin,
                       row_end, pos_row0, reinterpret_cast<const double2*>(pos), scale,
                       reinterpret_cast<double2*>(out));
    return (int)hipGetLastError();
}

extern "C" int cbf_euler(int32_t n, double* pos, const double* vel, double T, void* stream) {
    if (n < 0) return CBF_EINVAL;
    if (n == 0) return 0;
    if (!pos || !vel) return CBF_EINVAL;
    hipLaunchKernelGGL(k_euler, dim3(nblk(n)), dim3(kBlock), 0, (hipStream_t)stream, n,
                       reinterpret_cast<double2*>(pos), reinterpret_cast<const double2*>(vel), T);
    return (int)hipGetLastError();
}


extern "C" size_t cbf_lattice_workspace_size(int32_t W, int32_t win_rows, const cbf_grid* grid) {
    if (!grid || W <= 0 || win_rows <= 0 || grid->nx <= 0 || grid->ny <= 0) return 0;
    const long n = (long)W * win_rows;
    return CellWs::bytes(n, (long)grid->nx * grid->ny) + lattice_ext_bytes(n);
}


static int lattice_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                         int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                         double* vel_out, void* workspace, size_t workspace_bytes, unsigned long long* ext_keys,
                         ExtSpec X, void* stream) {
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    if (!vel_out) return CBF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * win_rows;
    const CellGrid G = make_grid(grid);
    CellWs Wk(workspace, n, (long)G.nx * G.ny);
    const double2* p2 = reinterpret_cast<const double2*>(pos);
    // unsharded: the window is the owned rows, so the nominal controls go straight to vel_out
    double2* wv = (win_row0 == row_begin && win_rows == row_end - row_begin) ? reinterpret_cast<double2*>(vel_out)
                                                                              : Wk.wvel;
    int3* bcs = reinterpret_cast<int3*>(Wk.cs);  // 12 B per agent (the area reserves 16)
    hipLaunchKernelGGL(k_lattice_nominal_bin_ordered, dim3(nblk(n)), dim3(kBlock), 0, s, G, W, H, row_begin, row_end,
                       win_row0, win_rows, p2, gain, wv, reinterpret_cast<double2*>(vel_out), Wk.count, Wk.sidx,
                       Wk.start, Wk.ncell, bcs, Wk.hardq, ext_keys, X, Wk.sctl);
    launch_scan(Wk, s);
    hipLaunchKernelGGL(k_lattice_scatter_ordered, dim3(nblk(n)), dim3(kBlock), 0, s, n, bcs, Wk.start, p2, wv, Wk.spos,
                       Wk.svel, Wk.sidx, Wk.spos32, Wk.hardq + 2, n, Wk.ncell, win_row0, H, W, row_begin, row_end, gain,
                       reinterpret_cast<double2*>(vel_out));
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                 int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                                 double* vel_out, void* workspace, size_t workspace_bytes, void* stream) {
    return lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                         workspace_bytes, nullptr, ExtSpec{0, 0, 0}, stream);
}

static int lattice_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                           int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                           double* pos_out, double* u, int32_t* status, int32_t* nbr_count, int32_t guard_rows,
                           double* extents, uint64_t* solves, void* workspace, size_t workspace_bytes,
                           int32_t cnt_begin, int32_t cnt_end, void* stream) {
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    if (!pos_out || !u || !status) return CBF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * win_rows;
    const CellGrid G = make_grid(grid);
    CellWs Wk(workspace, n, (long)G.nx * G.ny);
    double* ext_part = extents ? (double*)((char*)workspace + CellWs::bytes(n, Wk.ncell)) : nullptr;
    const int nb = nblk(n);
    const int hb = nb < kHardBlocks ? nb : kHardBlocks;
    const KP kp = make_kp(p);
    double2* po = reinterpret_cast<double2*>(pos_out);
    double2* uo = reinterpret_cast<double2*>(u);
    if (CBF_LDS_STAGE && !ext_part) {
        hipLaunchKernelGGL(p->f_is_zero ? k_lattice_filter_lds<true> : k_lattice_filter_lds<false>, dim3(nb),
                           dim3(kBlock), 0, s, kp, G, W, row_begin, row_end, win_row0, Wk.ncell, Wk.spos, Wk.svel,
                           Wk.sidx, Wk.start, T, po, uo, status, nbr_count,
                           reinterpret_cast<unsigned long long*>(solves), Wk.hardq, cnt_begin, cnt_end);
    } else {
        hipLaunchKernelGGL(p->f_is_zero ? k_lattice_filter<true> : k_lattice_filter<false>, dim3(nb), dim3(kBlock), 0,
                           s, kp, G, W, row_begin, row_end, win_row0, Wk.ncell, Wk.spos, Wk.svel, Wk.sidx, Wk.start, T,
                           po, uo, status, nbr_count, guard_rows, ext_part,
                           reinterpret_cast<unsigned long long*>(solves), Wk.hardq, Wk.spos32, cnt_begin, cnt_end);
    }
    // queue kernel only when the filter queues (CBF_HARD_INLINE solves hard QPs in place)
    const bool queued = !CBF_HARD_INLINE || CBF_HIT_MASK || (CBF_LDS_STAGE && !ext_part);
    if (queued)
        hipLaunchKernelGGL(k_lattice_filter_hard, dim3(hb), dim3(64), 0, s, kp, row_begin, row_end, T, po, uo, status,
                           nbr_count, guard_rows, ext_part ? ext_part + 4l * lattice_ext_waves(n) : nullptr,
                           Wk.hardq, (int)n);
    if (extents) launch_extents_finalize((int)lattice_ext_waves(n) + (queued ? hb : 0), ext_part, extents, s);
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                   int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                   const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                   int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* solves,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, extents, solves, workspace, workspace_bytes, row_begin, row_end, stream);
}

extern "C" int cbf_lattice_step(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                                double T, double* pos_out, double* vel_out, double* u, int32_t* status,
                                int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* solves,
                                void* workspace, size_t workspace_bytes, void* stream) {
    int rc = cbf_lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                               workspace_bytes, stream);
    if (rc) return rc;
    return cbf_lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status,
                               nbr_count, guard_rows, extents, solves, workspace, workspace_bytes, stream);
}

extern "C" int cbf_lattice_step_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                        int32_t row_begin, int32_t row_end, int32_t own_begin, int32_t own_end,
                                        int32_t win_row0, int32_t win_rows, const double* pos, double gain, double T,
                                        double* pos_out, double* vel_out, double* u, int32_t* status,
                                        int32_t* nbr_count, int32_t guard_rows, uint64_t* ext_keys, uint64_t* solves,
                                        void* workspace, size_t workspace_bytes, void* stream) {
    if (!ext_keys || guard_rows < 0 || own_begin < row_begin || own_end > row_end || own_begin >= own_end)
        return CBF_EINVAL;
    int rc = lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                           workspace_bytes, reinterpret_cast<unsigned long long*>(ext_keys),
                           ExtSpec{own_begin, own_end, guard_rows}, stream);
    if (rc) return rc;
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, nullptr, solves, workspace, workspace_bytes, own_begin, own_end, stream);
}

// ---- halo exchange of the row-sharded step -----------------------------------------
namespace {

__device__ __forceinline__ double dkey_inv(unsigned long long k) {
    const unsigned long long u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)u);
}

// send = [first halo rows | last halo rows | nsub records of 8 doubles (6 extents used)]; wave q
// of block 0 (q < nsub) reduces the 64 extent-key slots of sub-step q into its record and resets
// them for the next accumulation.
__global__ void __launch_bounds__(kBlock) k_halo_pack(int W, int halo, long n_own, const double2* __restrict__ own,
                                                      unsigned long long* __restrict__ keys, int nsub,
                                                      double* __restrict__ send) {
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const long rs = (long)halo * W;
    double2* s2 = reinterpret_cast<double2*>(send);
    if (t < rs) s2[t] = own[t];
    else if (t < 2 * rs) s2[t] = own[n_own - 2 * rs + t];
    if (blockIdx.x == 0) {
        const int l = threadIdx.x & 63;
        for (int q = threadIdx.x >> 6; q < nsub; q += kBlock / 64) {
            unsigned long long k[kExtVals];
#pragma unroll
            for (int v = 0; v < kExtVals; ++v) k[v] = dkey(ext_is_min(v) ? INFINITY : -INFINITY);
            for (int j = l; j < kExtSlots; j += 64) {
                unsigned long long* kl = keys + (long)kExtSlotWords * (kExtSlots * q + j);
#pragma unroll
                for (int v = 0; v < kExtVals; ++v) {
                    const unsigned long long x = kl[v];
                    k[v] = ext_is_min(v) ? (x < k[v] ? x : k[v]) : (x > k[v] ? x : k[v]);
                    kl[v] = dkey(ext_is_min(v) ? INFINITY : -INFINITY);
                }
            }
            for (int o = 32; o > 0; o >>= 1)
#pragma unroll
                for (int v = 0; v < kExtVals; ++v) {
                    const unsigned long long x = __shfl_xor(k[v], o, 64);
                    k[v] = ext_is_min(v) ? (x < k[v] ? x : k[v]) : (x > k[v] ? x : k[v]);
                }
            if (l == 0) {
                double* e = send + 4 * rs + 8 * q;
#pragma unroll
                for (int v = 0; v < kExtVals; ++v) e[v] = dkey_inv(k[v]);
            }
        }
    }
}

__global__ void k_ext_reset(unsigned long long* __restrict__ keys, int nsub) {
    for (int i = threadIdx.x; i < kExtSlots * nsub; i += blockDim.x) {
        unsigned long long* kl = keys + (long)kExtSlotWords * i;
#pragma unroll
        for (int v = 0; v < kExtVals; ++v) kl[v] = dkey(ext_is_min(v) ? INFINITY : -INFINITY);
    }
}

// Guard of one sub-step: every agent outside rank's candidate rows is farther than the cull
// radius (in y) from every agent rank computed.  Record layout (per rank q, per sub-step): {min y,
// max y of q's computed rows, max y of q's owned rows below its top `guard` rows, min y above its
// bottom `guard` rows, min y, max y of q's owned rows}.
__device__ __forceinline__ bool halo_guard_ok(const double* E, long stride, int ws, int rank, double radius) {
    const double rm = radius * (1.0 + 1e-9) + 1e-12;
    const double* me = E + (long)rank * stride;
    const double ymin = me[0], ymax = me[1];
    if (!(ymin <= ymax)) return true;  // no computed agents recorded (identity record)
    bool ok = true;
    for (int q = 0; q < ws; ++q) {
        const double* o = E + (long)q * stride;
        if (q < rank) {  // rows below: rank-1's rows outside our candidate band, all of lower ranks
            const double lim = (q == rank - 1) ? o[2] : o[5];
            if (!(ymin - lim > rm)) ok = false;
        } else if (q > rank) {
            const double lim = (q == rank + 1) ? o[3] : o[4];
            if (!(lim - ymax > rm)) ok = false;
        }
    }
    return ok;
}

// Window halo rows from the gathered slabs (rank-1's last rows below, rank+1's first rows above);
// block 0 lane 0 runs the guard on the gathered extents.
__global__ void __launch_bounds__(kBlock) k_halo_unpack(int W, int halo, int rows_lo, int rows_hi, long hi_off,
                                                        const double* __restrict__ recv, long stride, int ws, int rank,
                                                        double radius, int nsub, double2* __restrict__ wpos,
                                                        int32_t* __restrict__ flag) {
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const long nlo = (long)rows_lo * W, nhi = (long)rows_hi * W, rs = (long)halo * W;
    if (t < nlo) {
        const double2* src = reinterpret_cast<const double2*>(recv + (long)(rank - 1) * stride) + rs + (rs - nlo);
        wpos[t] = src[t];
    } else if (t < nlo + nhi) {
        const double2* src = reinterpret_cast<const double2*>(recv + (long)(rank + 1) * stride);
        wpos[hi_off + (t - nlo)] = src[t - nlo];
    }
    if (blockIdx.x == 0 && threadIdx.x < nsub && !halo_guard_ok(recv + 4 * rs + 8 * threadIdx.x, stride, ws, rank, radius))
        atomicOr(flag, 1);
}

}  // namespace

extern "C" size_t cbf_halo_ext_bytes(int32_t nsub) {
    return nsub < 1 ? 0 : (size_t)nsub * kExtSlots * kExtSlotWords * sizeof(unsigned long long);
}

extern "C" int cbf_halo_ext_reset(uint64_t* ext_keys, int32_t nsub, void* stream) {
    if (!ext_keys || nsub < 1) return CBF_EINVAL;
    hipLaunchKernelGGL(k_ext_reset, dim3(1), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<unsigned long long*>(ext_keys), nsub);
    return (int)hipGetLastError();
}

extern "C" int cbf_halo_pack(int32_t W, int32_t halo, int64_t n_own, const double* own, uint64_t* ext_keys,
                             int32_t nsub, double* send, void* stream) {
    if (W <= 0 || halo <= 0 || n_own < 2l * halo * W || !own || !ext_keys || !send || nsub < 1) return CBF_EINVAL;
    const long n = 2l * halo * W;
    hipLaunchKernelGGL(k_halo_pack, dim3(nblk(n)), dim3(kBlock), 0, (hipStream_t)stream, W, halo, (long)n_own,
                       reinterpret_cast<const double2*>(own), reinterpret_cast<unsigned long long*>(ext_keys), nsub,
                       send);
    return (int)hipGetLastError();
}

extern "C" int cbf_halo_unpack(int32_t W, int32_t halo, int32_t rows_lo, int32_t rows_hi, int64_t hi_row_offset,
                               const double* recv, int64_t stride, int32_t world_size, int32_t rank, double radius,
                               int32_t nsub, double* wpos, int32_t* flag, void* stream) {
    if (W <= 0 || halo <= 0 || rows_lo < 0 || rows_hi < 0 || rows_lo > halo || rows_hi > halo || !recv || !wpos ||
        !flag || world_size < 1 || rank < 0 || rank >= world_size || nsub < 1 || nsub > 64 ||
        stride < 4l * halo * W + 8l * nsub || (rows_lo > 0 && rank == 0) || (rows_hi > 0 && rank == world_size - 1) ||
        hi_row_offset < 0)
        return CBF_EINVAL;
    const long n = (long)(rows_lo + rows_hi) * W;
    hipLaunchKernelGGL(k_halo_unpack, dim3(nblk(n > 0 ? n : 1)), dim3(kBlock), 0, (hipStream_t)stream, W, halo,
                       rows_lo, rows_hi, (long)hi_row_offset * W, recv, (long)stride, world_size, rank, radius, nsub,
                       reinterpret_cast<double2*>(wpos), flag);
    return (int)hipGetLastError();
}
