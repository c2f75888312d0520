// swarm.hip -- nominal control, Euler, and the fused lattice-swarm timestep (gfx950).
//   graph-Laplacian consensus / cyclic pursuit   cross_and_rescue.py:108-125, meet_at_center.py:86-103
//   Euler                                        cross_and_rescue.py:173
//   whole timestep of a lattice swarm            SURVEY cfg3/cfg4 (cross_and_rescue.py:97-175 shape)
#include <hip/hip_ext.h>
#include "cbf_device.hpp"
#include "cells.hpp"
#include "lattice.hpp"
#include "lattice_ego.hpp"
#include "cbf_amd_measure.h"

using namespace cbf;

namespace {

inline int nblk(long n) { return (int)((n + kBlock - 1) / kBlock); }

// Chained binning: the build an advance bins its new positions for (the same window in
// cbf_lattice_run; the next sub-step's window, its own workspace, in cbf_lattice_cycle_sharded).
// Records are indexed by this advance's slots and name the agent by its index in the next window
// (= this window's index - shift), which holds exactly this advance's owned agents; an agent is
// binned (computable: its lattice neighbours are in the window) iff that index is in
// [comp_lo, comp_hi) (bounds, no division).  The next build's scatter computes its halo-guard
// extents (sharded), as the bin kernel does for an unchained build.
struct ChainSpec {
    int3* bcs;            // next build's records (null: no chaining)
    int32_t* count;       // next build's cell counts
    int32_t* sctl;        // next build's control words
    int shift, comp_lo, comp_hi;
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

// Lattice step K1, temporally coherent form: lanes walk the window agents in the previous step's
// cell order (identity on the first call), so consecutive lanes mostly share a cell; each run of
// equal cells in a wave takes its slots with ONE atomic (run length), and the later scatter
// writes nearly sequential slots.  Per-lane result bcs[t] = {cell, slot, agent} (12 B).
__global__ void __launch_bounds__(kBlock) k_lattice_nominal_bin_ordered(
    CellGrid G, int W, int H, int row_begin, int row_end, int win_row0, int win_rows, const double2* __restrict__ pos,
    int32_t* __restrict__ count, const int32_t* __restrict__ order, const int32_t* __restrict__ start, long ncell,
    int3* __restrict__ bcs, int32_t* __restrict__ hardq, unsigned long long* __restrict__ ext_keys, ExtSpec X,
    int32_t* __restrict__ sctl) {
    const long t = (long)xcd_block() * kBlock + threadIdx.x;
    const long nwin = (long)win_rows * W;
    if (t == 0) build_begin(sctl, nwin, ncell);
    __shared__ unsigned long long red[6][kBlock / 64];
    __shared__ int arrive;
    if (ext_keys) {
        if (threadIdx.x == 0) arrive = 0;
        __syncthreads();
    }
    // hardq[2..7]: the previous build left a cell order for exactly this window and grid (else
    // identity).  The order only permutes the work; it must list every window agent once, which
    // holds when window size, width, first row, lattice height and cell count all match.
    const bool ordered = hardq[2] == 1 && hardq[3] == (int)nwin && hardq[4] == (int)ncell && hardq[5] == win_row0 &&
                         hardq[6] == H && hardq[7] == W;
    int n_order = ordered ? start[ncell] : 0;
    n_order = n_order < 0 ? 0 : (n_order > nwin ? (int)nwin : n_order);
    int cell = -1;
    long w = -1;
    double2 p = make_double2(0.0, 0.0);
    if (t < nwin) {
        w = ordered ? (t < n_order ? order[t] : -1) : t;
        if (w >= 0 && w < nwin) {
            const int r = win_row0 + (int)(w / W);
            if ((r == 0 || r - 1 >= win_row0) && (r == H - 1 || r + 1 < win_row0 + win_rows)) {
                p = pos[w];
                cell = cell_of(G, p.x, p.y);
            }
        }
    }
    if (ext_keys) {
        // y-extents of the INPUT positions for the halo guard of the sharded step (checked at the
        // next exchange): {min, max} over the computed rows [row_begin, row_end), and over the
        // owned rows {max y of rows < own_end - guard, min y of rows >= own_begin + guard, min,
        // max}.  Reduced per block, then one atomic per value into one of 64 slots on separate
        // 128-B lines (cross-XCD atomics on a shared line serialise at the memory side).
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
        ext_keys_flush<kBlock / 64>(e, any, p.y, ext_keys, blockIdx.x, red, &arrive);
    }
    const int rank = run_rank(cell, count);
    if (t >= nwin) return;
    bcs[t] = cell < 0 ? make_int3(-1, 0, (int)w) : make_int3(cell, rank, (int)w);
}

#ifndef CBF_TILE_SPIN_LIMIT
#define CBF_TILE_SPIN_LIMIT (1l << 22)
#endif

// Logical block index of physical block b of nb (nb a multiple of 8 or not) with one contiguous
// range of logical blocks per XCD (xcd_block() for a sub-range of a grid that starts at an XCD
// boundary: physical block b runs on XCD b mod 8).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, rem = nb & 7, x = b & 7, j = b >> 3;
    return (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + j;
}

// Lattice build K2+K3, scan and scatter in one launch.  Blocks [0, ntiles) are the single-pass
// scan's tiles (scan_tile), each publishing a done word once its starts are written; blocks from
// ntiles8 (ntiles rounded up to the XCD count, so the scatter blocks keep their XCD-aware order)
// are the counting-sort scatter of the binned window agents into the cell-sorted copies, with each
// agent's lattice-Laplacian nominal control (cross_and_rescue.py:121-125 shape) computed on the
// way: the agent's position is loaded anyway and its 4 lattice neighbours are mostly L2 hits (cell
// order ~ lattice order), so the control never makes an HBM round trip.  A scatter thread takes
// CBF_SCATTER_A records (one per kBlock-wide sub-block, so every load stays coalesced) and issues
// ALL their loads -- records, positions, neighbours: the bulk of the scatter's memory traffic --
// before it waits, so that with CBF_SCATTER_A records per thread the whole scatter's grid fits on
// the chip at once and its loads overlap the scan (one record per thread left half the grid
// waiting for residency behind the scan: 22 us = scan + scatter back to back).  Then one lane per
// wave polls the done words of the tiles holding the wave's cells (the records arrive in the
// previous step's cell order, so they span one tile or two), and every lane reads its starts (sc1
// loads of write-through stores, scan_tile's hand-off) and stores.  Every wait points at a lower
// block index, which the dispatcher has already made resident (the single-pass scan relies on the
// same order).  A wait that runs out of spins sets the build's error flag (sctl[2], as a scan
// look-back that gives up); the filters then report CBF_STATUS_WORKSPACE_ERROR for the step, and
// the stores stay in bounds.
#ifndef CBF_SCATTER_A
#define CBF_SCATTER_A 2
#endif
constexpr int kScatterA = CBF_SCATTER_A;
__global__ void __launch_bounds__(kBlock) k_lattice_scan_scatter(
    int32_t* __restrict__ count, long ncell, int ntiles, int ntiles8, int32_t* __restrict__ start,
    unsigned long long* __restrict__ tstate, int32_t* __restrict__ tdone, int32_t* __restrict__ sctl, long nwin,
    long nrec, const int3* __restrict__ bcs, const double2* __restrict__ pos, double2* __restrict__ spos,
    double2* __restrict__ svel, int32_t* __restrict__ sidx, int32_t* __restrict__ order_state, int win_row0, int H,
    int W, int row_begin, int row_end, double gain, double2* __restrict__ vel_out,
    unsigned long long* __restrict__ ext_keys, ExtSpec X) {
    if ((int)blockIdx.x < ntiles8) {
        if ((int)blockIdx.x < ntiles) scan_tile(count, ncell, ntiles, start, tstate, sctl, blockIdx.x, tdone);
        return;
    }
    __shared__ unsigned long long red[6][kBlock / 64];
    __shared__ int arrive;
    if (ext_keys) {
        if (threadIdx.x == 0) arrive = 0;
        __syncthreads();
    }
    const int lb = xcd_remap((int)blockIdx.x - ntiles8, (int)gridDim.x - ntiles8);
    const long t0 = (long)lb * (kBlock * kScatterA) + threadIdx.x;
    const unsigned epoch = (unsigned)__hip_atomic_load(&sctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool usable = sctl[2] == 0;
    if (t0 == 0 && usable) {  // the cell order now exists for this window and grid: the next build walks it
        order_state[0] = 1;
        order_state[1] = (int)nwin;
        order_state[2] = (int)ncell;
        order_state[3] = win_row0;
        order_state[4] = H;
        order_state[5] = W;
    }
    const NominalSpec N = nominal_spec(sctl);
    int3 b[kScatterA];
    double2 p[kScatterA], u0[kScatterA];
    bool live[kScatterA];
#pragma unroll
    for (int a = 0; a < kScatterA; ++a) {
        const long t = t0 + (long)a * kBlock;
        b[a] = (t < nrec && usable) ? bcs[t] : make_int3(-1, 0, 0);
        live[a] = b[a].x >= 0 && b[a].x < ncell && b[a].z >= 0 && b[a].z < nwin;
    }
#pragma unroll
    for (int a = 0; a < kScatterA; ++a) {
        p[a] = make_double2(0.0, 0.0);
        u0[a] = make_double2(0.0, 0.0);
        if (live[a]) {
            const int z = b[a].z, r = win_row0 + z / W, c = z % W;
            p[a] = pos[z];
            if (N.mode == CBF_NOMINAL_RANDOM) {
                u0[a] = random_nominal(N, (long)win_row0 * W + z, p[a]);
            } else {
                const double2 s = lattice_sum(pos, z, r, c, W, H);
                u0[a] = make_double2(s.x * gain, s.y * gain);
            }
        }
    }
    // the wave's tiles: one lane polls their done words, then every lane reads the starts
    int tl = INT_MAX, th = -1;
#pragma unroll
    for (int a = 0; a < kScatterA; ++a)
        if (live[a]) {
            const int tt = b[a].x / kScanTile;
            tl = tt < tl ? tt : tl;
            th = tt > th ? tt : th;
        }
    const int tlo = wave_min_i(tl), thi = wave_max_i(th);
    if ((threadIdx.x & 63) == 0 && tlo <= thi) {
        const int32_t want = tile_done_word(epoch);
        bool failed = false;
        for (int tt = tlo; tt <= thi && !failed; ++tt) {
            long spins = 0;
            while (__hip_atomic_load(&tdone[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
                if (++spins > CBF_TILE_SPIN_LIMIT) {
                    __hip_atomic_store(&sctl[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    failed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    // the polling wave's loads of the handed-off words, all sc1, after its poll matched (scan_tile)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const bool ok = __hip_atomic_load(&sctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    int d[kScatterA];
#pragma unroll
    for (int a = 0; a < kScatterA; ++a)
        d[a] = (live[a] && ok) ? __hip_atomic_load(&start[b[a].x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + b[a].y
                               : -1;
    // halo-guard extents over the lane's agents; the maxima keep a NaN y (dkey orders it above +inf,
    // so it fails the guard, as with one agent per lane)
    double e[6] = {INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, -INFINITY};
    auto nmax = [](double m, double y) { return (y > m || y != y) ? y : m; };
    int any = 0;
    double py = 0.0;
#pragma unroll
    for (int a = 0; a < kScatterA; ++a) {
        if (!(d[a] >= 0 && d[a] < nwin)) continue;
        const int z = b[a].z, r = win_row0 + z / W, c = z % W;
        spos[d[a]] = p[a];
        svel[d[a]] = u0[a];
        if (vel_out && r >= row_begin && r < row_end) vel_out[(long)(r - row_begin) * W + c] = u0[a];
        sidx[d[a]] = z;
        if (ext_keys) {
            py = p[a].y;
            if (r >= row_begin && r < row_end) {
                e[0] = pmin(e[0], p[a].y);
                e[1] = nmax(e[1], p[a].y);
                any = 1;
            }
            if (r >= X.own_begin && r < X.own_end) {
                if (r < X.own_end - X.guard) e[2] = nmax(e[2], p[a].y);
                if (r >= X.own_begin + X.guard) e[3] = pmin(e[3], p[a].y);
                e[4] = pmin(e[4], p[a].y);
                e[5] = nmax(e[5], p[a].y);
                any = 1;
            }
        }
    }
    if (ext_keys) ext_keys_flush<kBlock / 64, kScatterA == 1>(e, any, py, ext_keys, lb, red, &arrive);
}

// Lattice step K4 for one cell-sorted slot: 3x3-cell cull (the three cell rows scanned as one
// sequence, hits compacted into the lane's LDS column), row assembly for the hits only (so
// divergent lanes do not pay assembly for every candidate iteration of the wave), then the tail.
// Rows are assembled as row_g and the quadrant terms added per quadrant (row_g's note); an ego
// whose quadrant terms are not all finite, or whose hit list overflowed, is assembled row by row
// with row_b (scan_range_direct).
template <bool FZ, bool ST, bool IN>
__device__ __forceinline__ void lattice_ego(const KP& P, const CellGrid& G, const WinBounds& B, int slot,
                                            const double2* __restrict__ spos, const double2* __restrict__ svel,
                                            const int32_t* __restrict__ sidx, const int32_t* __restrict__ start,
                                            double T, double2* __restrict__ pos_out, double2* __restrict__ u,
                                            int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                            int32_t* __restrict__ hardq, int q, HardRec* __restrict__ qrec, long qcap,
                                            int* hit_lds, Ego& E, EgoOut& O) {
    const int w = sidx[slot];
    O.w = w;
    if (!(w >= B.own_lo && w < B.own_hi)) return;
    const double2 pe = ld_slot(spos, slot), ve = ld_slot(svel, slot);
    ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    const int cx = cell_coord(pe.x, G.x0, G.inv_h, G.nx);
    const int cy = cell_coord(pe.y, G.y0, G.inv_h, G.ny);
    const int xa = cx > 0 ? cx - 1 : 0;
    const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
    int rt0[3], rt1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int yy = cy + k - 1;
        const bool in = yy >= 0 && yy < G.ny;
        rt0[k] = in ? start[yy * G.nx + xa] : 0;
        rt1[k] = in ? start[yy * G.nx + xb + 1] : 0;
    }
    HitList Hl;
    double d2 = INFINITY;
    scan_rows_joint(rt0, rt1, P, E, Hl, hit_lds, spos, d2);
    const double c0 = quad_c(P, E, 0), c1 = quad_c(P, E, 1), c2 = quad_c(P, E, 2), c3 = quad_c(P, E, 3);
    if (!Hl.overflowed() && isfinite(c0) && isfinite(c1) && isfinite(c2) && isfinite(c3)) {
        double* gq = reinterpret_cast<double*>(hit_lds + kHitCap * kBlock);
#pragma unroll
        for (int k = 0; k < 4; ++k) gq[k * kBlock + threadIdx.x] = INFINITY;
        Hl.template flush_gq<FZ>(hit_lds, gq, P, E, spos, svel);
        E.bq0 = gq[threadIdx.x] + c0;
        E.bq1 = gq[kBlock + threadIdx.x] + c1;
        E.bq2 = gq[2 * kBlock + threadIdx.x] + c2;
        E.bq3 = gq[3 * kBlock + threadIdx.x] + c3;
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) scan_range_direct<FZ>(rt0[k], rt1[k], P, E, spos, svel);
    }
    O.nbrs = E.count;
    if (ST) O.d2 = d2;
    ego_finish<FZ, ST, IN>(P, E, w, w - B.own_lo, slot, T, pos_out, u, status, cnt, hardq, q, qrec, qcap, O);
}

// K4: one lane per cell-sorted slot; QPs that solve_fast settles (the origin, or one Seidel event
// that stays put) are finished in place.  The others are solved right there by solve_ego (IN, the
// small-window instantiation) or appended with their assembled state to the hard queue for K5.
template <bool FZ, bool ST, bool IN>
__global__ void __launch_bounds__(kBlock) k_lattice_filter(KP P, CellGrid G, WinBounds B, int W, int row_begin,
                                                           int row_end, int win_row0, long nwin, long ncell,
                                                           const double2* __restrict__ spos,
                                                           const double2* __restrict__ svel,
                                                           const int32_t* __restrict__ sidx,
                                                           const int32_t* __restrict__ start,
                                                           const int32_t* __restrict__ sctl, double T,
                                                           double2* __restrict__ pos_out, double2* __restrict__ u,
                                                           int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                           double* __restrict__ ext_part,
                                                           unsigned long long* __restrict__ stats,
                                                           int32_t* __restrict__ hardq, HardRec* __restrict__ qrec,
                                                           long qcap, ChainSpec C) {
    // hit rows + 4 x fp64 per-quadrant minima, one column per lane
    __shared__ int hit_lds[kHitCap * kBlock + 8 * kBlock];
    const int bx = xcd_block();
    const int slot = bx * kBlock + threadIdx.x;
    if (IN) {
        // no queue kernel follows: a chained advance starts the next build's scan epoch here (an
        // error flag of this build stays set, so the rest of the run reports it; the scan reads the
        // epoch only after this kernel), and the last block refreshes the statistics snapshot
        // (values read mid-update are earlier ones, still valid lower bounds)
        if (C.bcs && bx == 0 && threadIdx.x == 0) {
            C.sctl[1] = (C.sctl[1] + 1) & 0x3FFFFFFF;
            if (C.sctl != sctl) C.sctl[2] = sctl[2];
        }
        if (ST && stats && (int)blockIdx.x == (int)gridDim.x - 1 && threadIdx.x < 64) stat_snapshot(stats);
    }
    if (sctl[2] != 0) {  // unusable cell list (build_begin / scan timeout): touch none of it
        lattice_error_tail(W, row_begin, row_end, win_row0, nwin, slot, u, status, cnt, stats, ext_part,
                           (long)bx * (kBlock / 64) + (threadIdx.x >> 6), hardq);
        return;
    }
    const int total = start[ncell];
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    EgoOut O;
    O.res = 0;
    O.w = -1;
    O.nbrs = 0;
    O.code = CBF_STATUS_IDLE;
    O.binding = false;
    O.seidel = false;
    O.viol = O.vorig = 0.0;
    O.d2 = INFINITY;
    Ego E;
    if (slot < total)  // finished (O.res == 1) or queued (O.res == 2)
        lattice_ego<FZ, ST, IN>(P, G, B, slot, spos, svel, sidx, start, T, pos_out, u, status, cnt, hardq,
                                bx % kSubQ, qrec, qcap, hit_lds, E, O);
    if (ext_part && O.res == 1) ext_accumulate_w(O.w, B, O.ny, e0, e1, e2, e3);
    if (C.bcs) {  // chained binning: the next build's record of this agent (queued egos: K5)
        // indexed by this advance's slot (the next scatter then reads its records in cell order and
        // writes nearly sequential slots); slots of agents outside the next window hold none
        const int wn = O.w - C.shift;
        const bool comp = O.res == 1 && wn >= C.comp_lo && wn < C.comp_hi;
        const int cell = comp ? cell_of(G, O.nx, O.ny) : -1;
        const int rank = run_rank(cell, C.count);
        if (slot < nwin && O.res != 2)
            C.bcs[slot] = comp ? make_int3(cell, rank, wn) : make_int3(-1, 0, O.res == 1 ? wn : -1);
    }
    if (ST && stats) {
        const bool counted = O.res != 0 && O.w >= B.cnt_lo && O.w < B.cnt_hi;
        wave_stats(stats, (long)bx * (kBlock / 64) + (threadIdx.x >> 6), counted && O.nbrs > 0,
                   counted && O.seidel, counted && O.res == 1, O.code, O.binding, O.viol, O.vorig,
                   counted ? O.d2 : INFINITY);
    }
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, (long)bx * (kBlock / 64) + (threadIdx.x >> 6));
}

// K5: the queued hard QPs (state assembled by K4): the exact Seidel solve, one per lane, the
// sub-queues drained in full waves (drain_subq).
__global__ void __launch_bounds__(64) k_lattice_filter_hard(KP P, CellGrid G, WinBounds B, double T,
                                                            double2* __restrict__ pos_out, double2* __restrict__ u,
                                                            int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                            double* __restrict__ ext_part,
                                                            unsigned long long* __restrict__ stats,
                                                            int32_t* __restrict__ hardq,
                                                            const HardRec* __restrict__ qrec, long qcap,
                                                            ChainSpec C, const int32_t* __restrict__ sctl) {
    // chained: the next build starts here (its bin kernel is skipped): advance the scan epoch; an
    // error flag of this build stays set, so the rest of the run reports it
    if (C.bcs && blockIdx.x == 0 && threadIdx.x == 0) {
        C.sctl[1] = (C.sctl[1] + 1) & 0x3FFFFFFF;
        if (C.sctl != sctl) C.sctl[2] = sctl[2];  // a failed build leaves the chained one unusable too
    }

    // the last block (idle unless its sub-queue is long) refreshes the statistics snapshot
    if (stats && blockIdx.x == gridDim.x - 1) stat_snapshot(stats);
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    int n_opt = 0, n_rel = 0, n_inf = 0, n_bnd = 0, n_sei = 0;
    double vo = 0.0, vr = 0.0;
    // the first block of each sub-queue (the one that works whenever it is non-empty) loads its
    // lane's first entry speculatively, beside the queue length (the queue area is allocated;
    // an entry past the length is never used): one memory round trip less before the solve
    const bool lead = (int)blockIdx.x < kSubQ;
    HardRec pre;
    if (lead) pre = qrec[(long)blockIdx.x * qcap + threadIdx.x];
    drain_subq(hardq, kHardPerQ, qcap, [&](int q, int i) {
        const HardRec h = (lead && i == (int)threadIdx.x) ? pre : qrec[(long)q * qcap + i];
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
        // CBF_STAT_SEIDEL counts the QPs that solve_fast cannot settle (the filter queues its
        // one-event QPs here too): statistics runs only
        if (stats && h.row >= B.cnt_lo && h.row < B.cnt_hi) {
            Sol S1;
            n_sei += solve_fast(P, E, S1) ? 0 : 1;
        }
        double ux, uy;
        clip_u(P, S, E, ux, uy);
        const double2 pn = make_double2(E.r0 + T * ux, E.r1 + T * uy);
        pos_out[h.k] = pn;
        if (u) u[h.k] = make_double2(ux, uy);
        if (status) status[h.k] = pack_status(S);
        if (cnt) cnt[h.k] = E.count;
        ext_accumulate_w(h.row, B, pn.y, e0, e1, e2, e3);
        if (C.bcs) {
            const int wn = h.row - C.shift;
            const bool comp = wn >= C.comp_lo && wn < C.comp_hi;
            const int cell = comp ? cell_of(G, pn.x, pn.y) : -1;
            C.bcs[h.slot] = comp ? make_int3(cell, atomicAdd(&C.count[cell], 1), wn) : make_int3(-1, 0, wn);
        }
        if (h.row >= B.cnt_lo && h.row < B.cnt_hi) {
            n_bnd += (S.x0 != 0.0 || S.x1 != 0.0) ? 1 : 0;
            if (S.status == CBF_STATUS_OPTIMAL) {
                ++n_opt;
                vo = pmax(vo, S.viol);
            } else if (S.status == CBF_STATUS_RELAXED) {
                ++n_rel;
                vr = pmax(vr, S.viol_orig);
            } else {
                ++n_inf;
            }
        }
    });
    if (stats) wave_stats_counts(stats, blockIdx.x, n_opt, n_rel, n_inf, n_bnd, n_sei, vo, vr);
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, blockIdx.x);
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


__global__ void k_set_nominal(int32_t* sctl, int mode, double amp, unsigned long long seed) {
    sctl[8] = mode;
    reinterpret_cast<double*>(sctl)[5] = amp;
    reinterpret_cast<unsigned long long*>(sctl)[6] = seed;
}

extern "C" int cbf_lattice_set_nominal(void* workspace, size_t workspace_bytes, int32_t mode, double amp,
                                       uint64_t seed, void* stream) {
    if (!workspace || workspace_bytes < 256) return CBF_EINVAL;
    if (mode != CBF_NOMINAL_CONSENSUS && mode != CBF_NOMINAL_RANDOM) return CBF_EINVAL;
    if (mode == CBF_NOMINAL_RANDOM && !(amp >= 0.0 && amp <= 1e300)) return CBF_EINVAL;
    hipLaunchKernelGGL(k_set_nominal, dim3(1), dim3(1), 0, (hipStream_t)stream, (int32_t*)workspace, (int)mode, amp,
                       (unsigned long long)seed);
    return (int)hipGetLastError();
}

extern "C" size_t cbf_lattice_workspace_size(int32_t W, int32_t win_rows, const cbf_grid* grid) {
    if (!grid || W <= 0 || win_rows <= 0 || grid->nx <= 0 || grid->ny <= 0) return 0;
    const long n = (long)W * win_rows;
    return CellWs::bytes(n, (long)grid->nx * grid->ny) + lattice_ext_bytes(n);
}


// the bin records, 12 B per agent (the cs area reserves 16)
static int3* lattice_bcs(const CellWs& Wk) { return reinterpret_cast<int3*>(Wk.cs); }

// scan + scatter (with the nominal control) of a build whose records are in lattice_bcs(Wk)
// nrec: records to read (the window of the binning pass: this build's own for the bin kernel, the
// previous sub-step's for a chained build, whose records are indexed by that advance's slots)
static void lattice_scan_scatter(const CellWs& Wk, int W, int H, int row_begin, int row_end, int win_row0, long n,
                                 const double2* pos, double gain, double* vel_out, hipStream_t s, long nrec = -1,
                                 unsigned long long* ext_keys = nullptr, ExtSpec X = ExtSpec{0, 0, 0}) {
    if (nrec < 0) nrec = n;
    const int ntiles8 = (Wk.ntiles + 7) & ~7;
    const int nsb = (int)((nrec + (long)kBlock * kScatterA - 1) / ((long)kBlock * kScatterA));
    hipLaunchKernelGGL(k_lattice_scan_scatter, dim3(ntiles8 + nsb), dim3(kBlock), 0, s, Wk.count, Wk.ncell,
                       Wk.ntiles, ntiles8, Wk.start, Wk.tstate, Wk.tdone, Wk.sctl, n, nrec, lattice_bcs(Wk),
                       pos, Wk.spos, Wk.svel, Wk.sidx, Wk.hardq + 2, win_row0, H, W, row_begin, row_end, gain,
                       reinterpret_cast<double2*>(vel_out), ext_keys, X);
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
    hipLaunchKernelGGL(k_lattice_nominal_bin_ordered, dim3(nblk(n)), dim3(kBlock), 0, s, G, W, H, row_begin, row_end,
                       win_row0, win_rows, p2, Wk.count, Wk.sidx, Wk.start, Wk.ncell, lattice_bcs(Wk), Wk.hardq,
                       ext_keys, X, Wk.sctl);
    lattice_scan_scatter(Wk, W, H, row_begin, row_end, win_row0, n, p2, gain, vel_out, s);
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                 int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                                 double* vel_out, void* workspace, size_t workspace_bytes, void* stream) {
    return lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                         workspace_bytes, nullptr, ExtSpec{0, 0, 0}, stream);
}

// The ChainSpec of the build of window rows [nw0, nw0 + nrows) in workspace nws, for an advance
// whose window starts at row w0.
static ChainSpec make_chain(const cbf_grid* grid, int W, int H, int w0, int nw0, int nrows, void* nws) {
    const long nn = (long)W * nrows;
    CellWs Nk(nws, nn, (long)grid->nx * grid->ny);
    ChainSpec C;
    C.bcs = lattice_bcs(Nk);
    C.count = Nk.count;
    C.sctl = Nk.sctl;
    C.shift = (nw0 - w0) * W;
    C.comp_lo = nw0 != 0 ? W : 0;                       // K1: the first window row only at the lattice edge
    C.comp_hi = nw0 + nrows != H ? (int)(nn - W) : (int)nn;  // ... the last likewise
    return C;
}

static int lattice_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                           int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                           double* pos_out, double* u, int32_t* status, int32_t* nbr_count, int32_t guard_rows,
                           double* extents, uint64_t* stats, void* workspace, size_t workspace_bytes,
                           int32_t cnt_begin, int32_t cnt_end, void* stream, const ChainSpec* chain = nullptr,
                           bool inner = false, hipEvent_t filter_done = nullptr,
                           hipEvent_t filter_start = nullptr) {
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    if (!pos_out || (!inner && (!u || !status))) return CBF_EINVAL;  // inner: a cbf_lattice_run timestep
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * win_rows;
    const CellGrid G = make_grid(grid);
    CellWs Wk(workspace, n, (long)G.nx * G.ny);
    double* ext_part = extents ? (double*)((char*)workspace + CellWs::bytes(n, Wk.ncell)) : nullptr;
    const int nb = nblk(n);
    const int hb = lattice_hard_blocks(n);
    const KP kp = make_kp(p);
    double2* po = reinterpret_cast<double2*>(pos_out);
    double2* uo = reinterpret_cast<double2*>(u);
    unsigned long long* st = reinterpret_cast<unsigned long long*>(stats);
    const WinBounds B = make_win_bounds(W, win_row0, n, row_begin, row_end, cnt_begin, cnt_end, guard_rows);
    // without a statistics array the filter is the instantiation that computes none of them
    // small windows (a few waves per SIMD, e.g. one stripe of a strong-scaled swarm): the
    // instantiation that runs the full solve in the filter itself -- its registers would halve the
    // big filter's occupancy, but a small window never fills the chip anyway -- and no queue kernel
    const bool in = solve_inline(p, n);
    const auto filter =
        in ? (st ? (p->f_is_zero ? k_lattice_filter<true, true, true> : k_lattice_filter<false, true, true>)
                 : (p->f_is_zero ? k_lattice_filter<true, false, true> : k_lattice_filter<false, false, true>))
           : (st ? (p->f_is_zero ? k_lattice_filter<true, true, false> : k_lattice_filter<false, true, false>)
                 : (p->f_is_zero ? k_lattice_filter<true, false, false> : k_lattice_filter<false, false, false>));
    if (filter_start) {  // the measurement hook: events carrying the filter dispatch's own start / end
        hipExtLaunchKernelGGL(filter, dim3(nb), dim3(kBlock), 0, s, filter_start, filter_done, 0u,
                              kp, G, B, W, row_begin, row_end, win_row0, n, Wk.ncell, Wk.spos, Wk.svel, Wk.sidx,
                              Wk.start, Wk.sctl, T, po, uo, status, nbr_count, ext_part, st, Wk.hardq, Wk.qrec,
                              Wk.qcap, chain ? *chain : ChainSpec{});
    } else {
        hipLaunchKernelGGL(filter, dim3(nb), dim3(kBlock), 0, s,
                           kp, G, B, W, row_begin, row_end, win_row0, n, Wk.ncell, Wk.spos, Wk.svel, Wk.sidx, Wk.start,
                           Wk.sctl, T, po, uo, status, nbr_count, ext_part, st, Wk.hardq, Wk.qrec, Wk.qcap,
                           chain ? *chain : ChainSpec{});
        if (filter_done)
            if (hipError_t e = hipEventRecord(filter_done, s)) return (int)e;
    }
    if (in) {
        if (extents) launch_extents_finalize((int)lattice_ext_waves(n), ext_part, extents, s);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_lattice_filter_hard, dim3(hb), dim3(64), 0, s,
                       kp, G, B, T, po, uo, status, nbr_count,
                       ext_part ? ext_part + 4l * lattice_ext_waves(n) : nullptr, st, Wk.hardq, Wk.qrec, Wk.qcap,
                       chain ? *chain : ChainSpec{}, Wk.sctl);
    if (extents) launch_extents_finalize((int)lattice_ext_waves(n) + hb, ext_part, extents, s);
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                   int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                   const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                   int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* stats,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, extents, stats, workspace, workspace_bytes, row_begin, row_end, stream);
}

extern "C" int cbf_lattice_solves_inline(const cbf_params* p, int64_t n) {
    return p && solve_inline(p, (long)n) ? 1 : 0;
}

extern "C" int cbf_lattice_advance_marked(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                          int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                          const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                          int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* stats,
                                          void* workspace, size_t workspace_bytes, void* filter_done, void* stream) {
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, extents, stats, workspace, workspace_bytes, row_begin, row_end, stream, nullptr,
                           false, (hipEvent_t)filter_done);
}

extern "C" int cbf_lattice_advance_timed(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                         int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                         const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                         int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* stats,
                                         void* workspace, size_t workspace_bytes, void* filter_start,
                                         void* filter_stop, void* stream) {
    if (!filter_start || !filter_stop) return CBF_EINVAL;
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, extents, stats, workspace, workspace_bytes, row_begin, row_end, stream, nullptr,
                           false, (hipEvent_t)filter_stop, (hipEvent_t)filter_start);
}

extern "C" int cbf_lattice_step(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                                int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double gain,
                                double T, double* pos_out, double* vel_out, double* u, int32_t* status,
                                int32_t* nbr_count, int32_t guard_rows, double* extents, uint64_t* stats,
                                void* workspace, size_t workspace_bytes, void* stream) {
    int rc = cbf_lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                               workspace_bytes, stream);
    if (rc) return rc;
    return cbf_lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status,
                               nbr_count, guard_rows, extents, stats, workspace, workspace_bytes, stream);
}

// The queued-QP kernel of an advance without chained binning (window cull): the egos of window
// bounds B, n window agents.
static void launch_hard_plain(const cbf_params* p, const cbf_grid* grid, const CellWs& Wk, const WinBounds& B, long n,
                              double T, double2* pos_out, double2* u, int32_t* status, int32_t* cnt,
                              unsigned long long* stats, hipStream_t s) {
    hipLaunchKernelGGL(k_lattice_filter_hard, dim3(lattice_hard_blocks(n)), dim3(64), 0, s, make_kp(p),
                       make_grid(grid), B, T, pos_out, u, status, cnt, (double*)nullptr, stats, Wk.hardq, Wk.qrec,
                       Wk.qcap, ChainSpec{}, Wk.sctl);
}
static void launch_hard_plain(const cbf_params* p, const cbf_grid* grid, const CellWs& Wk, int W, int H, double T,
                              double2* pos_out, double2* u, int32_t* status, int32_t* cnt, unsigned long long* stats,
                              hipStream_t s) {
    const long n = (long)W * H;
    launch_hard_plain(p, grid, Wk, make_win_bounds(W, 0, n, 0, H, 0, H, 0), n, T, pos_out, u, status, cnt, stats, s);
}

// cbf_lattice_run_ex with CBF_RUN_WINDOW_CULL: per timestep the window build (k_window_prep:
// nominal controls and the guards), the window filter and, for a large window, the queued-QP
// kernel.  The filter reads its input positions while writing new ones, so timesteps alternate
// between pos and the workspace's spos: with an odd count the first build also copies pos to spos
// and the first filter reads that copy, so the last timestep always writes pos.
static int lattice_run_window(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, double* pos,
                              double gain, double T, int32_t steps, double* vel_out, double* u, int32_t* status,
                              int32_t* nbr_count, uint64_t* stats, void* workspace, bool hist, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * H;
    CellWs Wk(workspace, n, (long)grid->nx * grid->ny);
    if (!window_cull_ok(W, H, n, Wk)) return CBF_EINVAL;
    const bool in = solve_inline(p, n);
    double2* buf[2] = {reinterpret_cast<double2*>(pos), Wk.spos};
    const int odd = steps & 1;
    unsigned long long* st = reinterpret_cast<unsigned long long*>(stats);
    for (int k = 0; k < steps; ++k) {
        double2* src = buf[(k + odd) & 1];
        double2* dst = buf[(k + 1 + odd) & 1];
        const bool last = k + 1 == steps, out = last || hist;
        const long o = hist ? (long)k * n : 0;
        // an odd run's first build reads pos and leaves its copy in spos, which the filter then reads
        const WinGeom Q = whole_lattice(W, H);
        window_prep(Wk, Q, k == 0 && odd ? buf[0] : src, gain, out ? reinterpret_cast<double2*>(vel_out) + o : nullptr,
                    k == 0 && odd ? buf[1] : nullptr, nullptr, 0, H, ExtSpec{0, 0, 0}, window_fold(p), s);
        double2* uo = out ? reinterpret_cast<double2*>(u) + o : nullptr;
        int32_t* so = out ? status + o : nullptr;
        int32_t* co = out && nbr_count ? nbr_count + o : nullptr;
        window_filter(p, Wk, Q, 0, H, 0, H, src, T, dst, uo, so, co, st, in, s);
        if (!in) launch_hard_plain(p, grid, Wk, W, H, T, dst, uo, so, co, st, s);
        if (int rc = (int)hipGetLastError()) return rc;
    }
    return 0;
}

// The two phases of one window-cull timestep as separate calls (the measurement hooks: the bench
// times the filter kernel alone), for the owned rows [row_begin, row_end) of a window of win_rows
// lattice rows from win_row0 (the whole lattice, or a sharded sub-step's window).  pos_out (index
// (r - row_begin) W + c) must not overlap pos.
static WinGeom window_geom(int W, int H, int win_row0, int win_rows) {
    return WinGeom{W, win_rows, win_row0, H, win_row0 > 0 ? 1 : 0,
                   win_row0 + win_rows < H ? win_rows - 1 : win_rows};
}

extern "C" int cbf_lattice_window_build_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                           int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                           const double* pos, double gain, double* vel_out, void* workspace,
                                           size_t workspace_bytes, void* stream) {
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    const long n = (long)W * win_rows;
    CellWs Wk(workspace, n, (long)grid->nx * grid->ny);
    if (!window_cull_ok(W, win_rows, n, Wk)) return CBF_EINVAL;
    window_prep(Wk, window_geom(W, H, win_row0, win_rows), reinterpret_cast<const double2*>(pos), gain,
                reinterpret_cast<double2*>(vel_out), nullptr, nullptr, row_begin, row_end, ExtSpec{0, 0, 0},
                window_fold(p), (hipStream_t)stream);
    return (int)hipGetLastError();
}

static int window_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                          int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                          double* pos_out, double* u, int32_t* status, int32_t* nbr_count, uint64_t* stats,
                          void* workspace, size_t workspace_bytes, hipEvent_t filter_done, hipEvent_t filter_start,
                          void* stream) {
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    const long n = (long)W * win_rows, nown = (long)W * (row_end - row_begin);
    if (!pos_out || !u || !status) return CBF_EINVAL;
    if (pos_out < pos + 2 * n && pos < pos_out + 2 * nown) return CBF_EINVAL;  // the filter reads pos throughout
    CellWs Wk(workspace, n, (long)grid->nx * grid->ny);
    if (!window_cull_ok(W, win_rows, n, Wk)) return CBF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const bool in = solve_inline(p, n);
    double2* po = reinterpret_cast<double2*>(pos_out);
    double2* uo = reinterpret_cast<double2*>(u);
    unsigned long long* st = reinterpret_cast<unsigned long long*>(stats);
    window_filter(p, Wk, window_geom(W, H, win_row0, win_rows), row_begin, row_end, row_begin, row_end,
                  reinterpret_cast<const double2*>(pos), T, po, uo, status, nbr_count, st, in, s, filter_start,
                  filter_start ? filter_done : nullptr);
    if (filter_done && !filter_start)
        if (hipError_t e = hipEventRecord(filter_done, s)) return (int)e;
    if (!in)
        launch_hard_plain(p, grid, Wk, make_win_bounds(W, win_row0, n, row_begin, row_end, row_begin, row_end, 0), n,
                          T, po, uo, status, nbr_count, st, s);
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_window_advance_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                             int32_t row_begin, int32_t row_end, int32_t win_row0, int32_t win_rows,
                                             const double* pos, double T, double* pos_out, double* u,
                                             int32_t* status, int32_t* nbr_count, uint64_t* stats, void* workspace,
                                             size_t workspace_bytes, void* filter_done, void* stream) {
    return window_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                          stats, workspace, workspace_bytes, (hipEvent_t)filter_done, nullptr, stream);
}

extern "C" int cbf_lattice_window_advance_timed(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                                const double* pos, double T, double* pos_out, double* u,
                                                int32_t* status, int32_t* nbr_count, uint64_t* stats,
                                                void* workspace, size_t workspace_bytes, void* filter_start,
                                                void* filter_stop, void* stream) {
    if (!filter_start || !filter_stop) return CBF_EINVAL;
    return window_advance(p, grid, W, H, 0, H, 0, H, pos, T, pos_out, u, status, nbr_count, stats, workspace,
                          workspace_bytes, (hipEvent_t)filter_stop, (hipEvent_t)filter_start, stream);
}

extern "C" int cbf_lattice_window_counters(const void* workspace, size_t workspace_bytes, uint64_t* out,
                                           void* stream) {
    return window_counters(workspace, workspace_bytes, out, (hipStream_t)stream);
}

extern "C" int cbf_lattice_window_build(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                        const double* pos, double gain, double* vel_out, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    return cbf_lattice_window_build_ex(p, grid, W, H, 0, H, 0, H, pos, gain, vel_out, workspace, workspace_bytes,
                                       stream);
}

extern "C" int cbf_lattice_window_advance(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                          const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                          int32_t* nbr_count, uint64_t* stats, void* workspace,
                                          size_t workspace_bytes, void* filter_done, void* stream) {
    return cbf_lattice_window_advance_ex(p, grid, W, H, 0, H, 0, H, pos, T, pos_out, u, status, nbr_count, stats,
                                         workspace, workspace_bytes, filter_done, stream);
}

// `steps` timesteps of the whole lattice in one call, bit-identical to as many cbf_lattice_step
// calls: every advance but the last bins its new positions for the next build on the fly
// (chained binning: run_rank in K4, one atomic per queued ego in K5), so only the first build
// runs the bin kernel.  Positions, workspace and stats as cbf_lattice_step; vel_out, u, status
// and nbr_count hold the last step's.
extern "C" int cbf_lattice_run_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, double* pos,
                                  double gain, double T, int32_t steps, double* vel_out, double* u, int32_t* status,
                                  int32_t* nbr_count, uint64_t* stats, void* workspace, size_t workspace_bytes,
                                  uint32_t flags, void* stream) {
    int rc = check_lattice(p, grid, W, H, 0, H, 0, H, pos, workspace, workspace_bytes);
    if (rc) return rc;
    if (steps < 0 || !vel_out || !u || !status || (flags & ~(CBF_RUN_OUTPUT_HISTORY | CBF_RUN_WINDOW_CULL)))
        return CBF_EINVAL;
    const bool hist = (flags & CBF_RUN_OUTPUT_HISTORY) != 0;
    if (flags & CBF_RUN_WINDOW_CULL)
        return lattice_run_window(p, grid, W, H, pos, gain, T, steps, vel_out, u, status, nbr_count, stats, workspace,
                                  hist, stream);
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * H;
    CellWs Wk(workspace, n, (long)grid->nx * grid->ny);
    const CellGrid G = make_grid(grid);
    const double2* p2 = reinterpret_cast<const double2*>(pos);
    for (int k = 0; k < steps; ++k) {
        if (k == 0)
            hipLaunchKernelGGL(k_lattice_nominal_bin_ordered, dim3(nblk(n)), dim3(kBlock), 0, s, G, W, H, 0, H, 0, H,
                               p2, Wk.count, Wk.sidx, Wk.start, Wk.ncell, lattice_bcs(Wk), Wk.hardq,
                               (unsigned long long*)nullptr, ExtSpec{0, 0, 0}, Wk.sctl);
        // vel_out, u, status and nbr_count are written by the last timestep only (the inner ones'
        // would be overwritten), or by every timestep into its slice of the history arrays
        const bool last = k + 1 == steps, out = last || hist;
        const long o = hist ? (long)k * n : 0;
        lattice_scan_scatter(Wk, W, H, 0, H, 0, n, p2, gain, out ? vel_out + 2 * o : nullptr, s);
        rc = (int)hipGetLastError();
        if (rc) return rc;
        const ChainSpec C = make_chain(grid, W, H, 0, 0, H, workspace);
        rc = lattice_advance(p, grid, W, H, 0, H, 0, H, pos, T, pos, out ? u + 2 * o : nullptr,
                             out ? status + o : nullptr, out && nbr_count ? nbr_count + o : nullptr, 0, nullptr,
                             stats, workspace, workspace_bytes, 0, H, stream, last ? nullptr : &C, !out);
        if (rc) return rc;
    }
    return 0;
}

extern "C" int cbf_lattice_run(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, double* pos,
                               double gain, double T, int32_t steps, double* vel_out, double* u, int32_t* status,
                               int32_t* nbr_count, uint64_t* stats, void* workspace, size_t workspace_bytes,
                               void* stream) {
    return cbf_lattice_run_ex(p, grid, W, H, pos, gain, T, steps, vel_out, u, status, nbr_count, stats, workspace,
                              workspace_bytes, 0u, stream);
}

// One exchange cycle of the row-sharded step (cbf_amd/shard.py): nsub sub-steps after the caller's
// halo unpack, sub-step s with workspace s of `workspaces` (nsub x ws_bytes).  Sub-step 0 builds
// its cell list from the window positions (bin kernel, guard extents of set 0); every advance but
// the last bins the rows it computed straight into the next sub-step's build (whose window is
// exactly those rows) and accumulates that build's guard extents.  Bit-identical to nsub
// cbf_lattice_step_sharded calls with the same geometry.
static int cycle_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t own_begin,
                         int32_t own_end, int32_t halo, int32_t nsub, int32_t sub_begin, int32_t sub_end,
                         int32_t win_row0, int32_t win_rows, double* wpos, double gain, double T, double* wvel,
                         double* wu, int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                         void* workspaces, size_t ws_bytes, bool window, void* stream);

extern "C" int cbf_lattice_cycle_sharded_ex(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                            int32_t own_begin, int32_t own_end, int32_t halo, int32_t nsub,
                                            int32_t sub_begin, int32_t sub_end, int32_t win_row0, int32_t win_rows,
                                            double* wpos, double gain, double T, double* wvel, double* wu,
                                            int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                                            void* workspaces, size_t ws_bytes, uint32_t flags, void* stream) {
    if (flags & ~CBF_RUN_WINDOW_CULL) return CBF_EINVAL;
    return cycle_sharded(p, grid, W, H, own_begin, own_end, halo, nsub, sub_begin, sub_end, win_row0, win_rows, wpos,
                         gain, T, wvel, wu, wstatus, wcnt, ext_keys, stats, workspaces, ws_bytes,
                         (flags & CBF_RUN_WINDOW_CULL) != 0, stream);
}

extern "C" int cbf_lattice_cycle_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                         int32_t own_begin, int32_t own_end, int32_t halo, int32_t nsub,
                                         int32_t sub_begin, int32_t sub_end,
                                         int32_t win_row0, int32_t win_rows, double* wpos, double gain, double T,
                                         double* wvel, double* wu, int32_t* wstatus, int32_t* wcnt,
                                         uint64_t* ext_keys, uint64_t* stats, void* workspaces, size_t ws_bytes,
                                         void* stream) {
    return cycle_sharded(p, grid, W, H, own_begin, own_end, halo, nsub, sub_begin, sub_end, win_row0, win_rows, wpos,
                         gain, T, wvel, wu, wstatus, wcnt, ext_keys, stats, workspaces, ws_bytes, false, stream);
}

// The window-cull form of an exchange cycle: per sub-step the window build (nominal controls,
// guards, and the halo-guard extents of its input, as the cell-list bin / scatter accumulate them),
// the window filter and the queued-QP kernel.  Sub-step s reads its window from one buffer and
// writes the rows it computes -- exactly the next sub-step's window -- to the other: wpos and
// workspace 0's spos (sized for the whole cycle window), so that the call's last sub-step writes
// wpos (with an odd count the first build copies its window to spos).  Same results as the
// cell-list cycle whenever its halo guard holds (the guard is the same).
template <class Sub>
static int cycle_sharded_window(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t own_begin,
                                int32_t own_end, int32_t nsub, int32_t sub_begin, int32_t sub_end, int32_t win_row0,
                                int32_t win_rows, double* wpos, double gain, double T, double* wvel, double* wu,
                                int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                                void* workspaces, size_t ws_bytes, Sub&& sub, hipStream_t st) {
    const long ncell = (long)grid->nx * grid->ny;
    const CellWs W0(workspaces, (long)W * win_rows, ncell);
    if (!window_cull_ok(W, win_rows, (long)W * win_rows, W0)) return CBF_EINVAL;
    double2* buf[2] = {reinterpret_cast<double2*>(wpos), W0.spos};
    const int n = sub_end - sub_begin, odd = n & 1;
    const size_t set_words = cbf_halo_ext_bytes(1) / 8;
    unsigned long long* stw = reinterpret_cast<unsigned long long*>(stats);
    for (int j = 0; j < n; ++j) {
        const int k = sub_begin + j;
        int a, b, sw0, sw1, guard;
        sub(k, a, b, sw0, sw1, guard);
        const int rows = sw1 - sw0;
        void* ws = (char*)workspaces + (size_t)k * ws_bytes;
        int rc = check_lattice(p, grid, W, H, a, b, sw0, rows, wpos, ws, ws_bytes);
        if (rc) return rc;
        const CellWs Wk(ws, (long)W * rows, ncell);
        if (!window_cull_ok(W, rows, (long)W * rows, Wk)) return CBF_EINVAL;
        const WinGeom Q{W, rows, sw0, H, sw0 > 0 ? 1 : 0, sw1 < H ? rows - 1 : rows};
        double2* src = buf[(j + odd) & 1] + (long)(sw0 - win_row0) * W;
        double2* dst = buf[(j + 1 + odd) & 1] + (long)(a - win_row0) * W;
        const bool last = j + 1 == n;
        const long o = (long)(a - win_row0) * W;
        unsigned long long* ek = reinterpret_cast<unsigned long long*>(ext_keys) + (size_t)k * set_words;
        // an odd call's first build reads wpos and leaves the copy its filter reads in spos
        window_prep(Wk, Q, j == 0 && odd ? buf[0] + (long)(sw0 - win_row0) * W : src, gain,
                    last ? reinterpret_cast<double2*>(wvel) + o : nullptr, j == 0 && odd ? src : nullptr, ek, a, b,
                    ExtSpec{own_begin, own_end, guard}, window_fold(p), st);
        double2* uo = last ? reinterpret_cast<double2*>(wu) + o : nullptr;
        int32_t* so = last ? wstatus + o : nullptr;
        int32_t* co = last && wcnt ? wcnt + o : nullptr;
        const bool in = solve_inline(p, (long)W * rows);
        window_filter(p, Wk, Q, a, b, own_begin, own_end, src, T, dst, uo, so, co, stw, in, st);
        if (!in)
            launch_hard_plain(p, grid, Wk, make_win_bounds(W, sw0, (long)W * rows, a, b, own_begin, own_end, 0),
                              (long)W * rows, T, dst, uo, so, co, stw, st);
        if (int e = (int)hipGetLastError()) return e;
    }
    return 0;
}

static int cycle_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t own_begin,
                         int32_t own_end, int32_t halo, int32_t nsub, int32_t sub_begin, int32_t sub_end,
                         int32_t win_row0, int32_t win_rows, double* wpos, double gain, double T, double* wvel,
                         double* wu, int32_t* wstatus, int32_t* wcnt, uint64_t* ext_keys, uint64_t* stats,
                         void* workspaces, size_t ws_bytes, bool window, void* stream) {
    if (!p || !grid || W <= 0 || H <= 0 || halo < 2 || nsub < 1 || own_begin < 0 || own_end > H ||
        own_begin >= own_end || sub_begin < 0 || sub_end > nsub || sub_begin >= sub_end)
        return CBF_EINVAL;
    const long G = (long)halo * nsub;
    if (G > own_end - own_begin) return CBF_EINVAL;
    const int w0 = (int)(own_begin - G > 0 ? own_begin - G : 0), w1 = (int)(own_end + G < H ? own_end + G : H);
    if (win_row0 != w0 || win_rows != w1 - w0) return CBF_EINVAL;
    if (!wpos || !wvel || !wu || !wstatus || !ext_keys || !workspaces) return CBF_EINVAL;
    if (ws_bytes < cbf_lattice_workspace_size(W, win_rows, grid)) return CBF_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const size_t set_words = cbf_halo_ext_bytes(1) / 8;
    auto sub = [&](int k, int& a, int& b, int& sw0, int& sw1, int& guard) {
        const int d = (int)G - halo * (k + 1);
        a = own_begin - d > 0 ? own_begin - d : 0;
        b = own_end + d < H ? own_end + d : H;
        sw0 = a - halo > 0 ? a - halo : 0;
        sw1 = b + halo < H ? b + halo : H;
        guard = d + halo - 1;
    };
    // a chained build's records are indexed by the previous sub-step's slots (12 B each; that
    // window has up to 2 halo rows more): they must fit its record area (16 B per agent of its
    // own window), which holds for stripes of >= 4 halo rows; checked before anything is launched
    for (int k = 1; k < nsub; ++k) {
        int a, b, w0k, w1k, g, pa, pb, pw0, pw1, pg;
        sub(k, a, b, w0k, w1k, g);
        sub(k - 1, pa, pb, pw0, pw1, pg);
        if (12l * (pw1 - pw0) > 16l * (w1k - w0k)) return CBF_EINVAL;
    }
    if (window)
        return cycle_sharded_window(p, grid, W, H, own_begin, own_end, nsub, sub_begin, sub_end, win_row0, win_rows,
                                    wpos, gain, T, wvel, wu, wstatus, wcnt, ext_keys, stats, workspaces, ws_bytes,
                                    sub, st);
    for (int k = sub_begin; k < sub_end; ++k) {
        int a, b, sw0, sw1, guard;
        sub(k, a, b, sw0, sw1, guard);
        void* ws = (char*)workspaces + (size_t)k * ws_bytes;
        // the per-sub-step outputs (nominal / filtered control, status, count) are written by the
        // call's last sub-step only: the earlier ones' would be overwritten there (its computed rows
        // contain the owned rows; the ghost rows' are not outputs)
        const bool last = k + 1 == sub_end;
        double* spos = wpos + 2l * (sw0 - win_row0) * W;
        const long o = (long)(a - win_row0) * W;
        unsigned long long* ek = reinterpret_cast<unsigned long long*>(ext_keys) + (size_t)k * set_words;
        int rc;
        if (k == sub_begin) {
            rc = lattice_build(p, grid, W, H, a, b, sw0, sw1 - sw0, spos, gain, wvel + 2 * o, ws, ws_bytes, ek,
                               ExtSpec{own_begin, own_end, guard}, stream);  // (vel_out: the bin build must)
        } else {
            rc = check_lattice(p, grid, W, H, a, b, sw0, sw1 - sw0, spos, ws, ws_bytes);
            if (!rc) {
                int pa, pb, pw0, pw1, pg;
                sub(k - 1, pa, pb, pw0, pw1, pg);
                const long n = (long)W * (sw1 - sw0), nprev = (long)W * (pw1 - pw0);
                CellWs Wk(ws, n, (long)grid->nx * grid->ny);
                lattice_scan_scatter(Wk, W, H, a, b, sw0, n, reinterpret_cast<const double2*>(spos), gain,
                                     last ? wvel + 2 * o : nullptr, st, nprev, ek, ExtSpec{own_begin, own_end, guard});
                rc = (int)hipGetLastError();
            }
        }
        if (rc) return rc;
        ChainSpec C;
        if (!last) {
            int na, nb, nw0, nw1, ng;
            sub(k + 1, na, nb, nw0, nw1, ng);
            C = make_chain(grid, W, H, sw0, nw0, nw1 - nw0, (char*)workspaces + (size_t)(k + 1) * ws_bytes);
        }
        rc = lattice_advance(p, grid, W, H, a, b, sw0, sw1 - sw0, spos, T, wpos + 2 * o, last ? wu + 2 * o : nullptr,
                             last ? wstatus + o : nullptr, last && wcnt ? wcnt + o : nullptr, guard, nullptr, stats, ws,
                             ws_bytes, own_begin, own_end, stream, last ? nullptr : &C, !last);
        if (rc) return rc;
    }
    return 0;
}

extern "C" int cbf_lattice_step_sharded(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                        int32_t row_begin, int32_t row_end, int32_t own_begin, int32_t own_end,
                                        int32_t win_row0, int32_t win_rows, const double* pos, double gain, double T,
                                        double* pos_out, double* vel_out, double* u, int32_t* status,
                                        int32_t* nbr_count, int32_t guard_rows, uint64_t* ext_keys, uint64_t* stats,
                                        void* workspace, size_t workspace_bytes, void* stream) {
    if (!ext_keys || guard_rows < 0 || own_begin < row_begin || own_end > row_end || own_begin >= own_end)
        return CBF_EINVAL;
    int rc = lattice_build(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, gain, vel_out, workspace,
                           workspace_bytes, reinterpret_cast<unsigned long long*>(ext_keys),
                           ExtSpec{own_begin, own_end, guard_rows}, stream);
    if (rc) return rc;
    return lattice_advance(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, T, pos_out, u, status, nbr_count,
                           guard_rows, nullptr, stats, workspace, workspace_bytes, own_begin, own_end, stream);
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

// ---- neighbour exchange (one all_to_all_single): rank r sends its first G rows to r-1 and its
// last G rows to r+1 only, and its nsub guard records (8 doubles each) to every rank, which the
// guard needs from all of them.  Chunk q of the send buffer (to rank q) and of the receive buffer
// (from rank q) are [records (8 nsub) | rows (G W double2s) if q = r +- 1]: the two layouts have the
// same sizes, so one offset formula serves both (cbf_amd/shard.py: ShardedLattice.nbr_splits).
__device__ __forceinline__ long nbr_chunk_off(int q, int rank, int ws, long r8, long rs2) {
    long o = (long)q * r8;
    if (rank > 0 && q > rank - 1) o += rs2;
    if (rank + 1 < ws && q > rank + 1) o += rs2;
    return o;
}

// rows: thread t < n_lo copies the first G rows (to rank - 1), the next n_hi the last G rows (to
// rank + 1); block 0 reduces the guard records as k_halo_pack does and writes them into every chunk
__global__ void __launch_bounds__(kBlock) k_halo_pack_nbr(int W, int halo, long n_own, const double2* __restrict__ own,
                                                          unsigned long long* __restrict__ keys, int nsub, int ws,
                                                          int rank, double* __restrict__ send) {
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const long rs = (long)halo * W, r8 = 8l * nsub;
    const long n_lo = rank > 0 ? rs : 0, n_hi = rank + 1 < ws ? rs : 0;
    if (t < n_lo) {
        reinterpret_cast<double2*>(send + nbr_chunk_off(rank - 1, rank, ws, r8, 2 * rs) + r8)[t] = own[t];
    } else if (t < n_lo + n_hi) {
        const long i = t - n_lo;
        reinterpret_cast<double2*>(send + nbr_chunk_off(rank + 1, rank, ws, r8, 2 * rs) + r8)[i] = own[n_own - rs + i];
    }
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
            // lane d writes the record into the chunks of destinations d, d + 64, ...
            for (int d = l; d < ws; d += 64) {
                double* e = send + nbr_chunk_off(d, rank, ws, r8, 2 * rs) + 8 * q;
#pragma unroll
                for (int v = 0; v < kExtVals; ++v) e[v] = dkey_inv(k[v]);
            }
        }
    }
}

// the guard of one sub-step over records at recv + off(q) + 8 s (halo_guard_ok's rule)
__device__ __forceinline__ bool halo_guard_ok_nbr(const double* recv, int s, int ws, int rank, long r8, long rs2,
                                                  double radius) {
    const double rm = radius * (1.0 + 1e-9) + 1e-12;
    const double* me = recv + nbr_chunk_off(rank, rank, ws, r8, rs2) + 8 * s;
    const double ymin = me[0], ymax = me[1];
    if (!(ymin <= ymax)) return true;
    bool ok = true;
    for (int q = 0; q < ws; ++q) {
        const double* o = recv + nbr_chunk_off(q, rank, ws, r8, rs2) + 8 * s;
        if (q < rank) {
            const double lim = (q == rank - 1) ? o[2] : o[5];
            if (!(ymin - lim > rm)) ok = false;
        } else if (q > rank) {
            const double lim = (q == rank + 1) ? o[3] : o[4];
            if (!(lim - ymax > rm)) ok = false;
        }
    }
    return ok;
}

// Window ghost rows from the neighbours' chunks (rank-1's last rows_lo rows below, rank+1's first
// rows_hi rows above); block 0 lanes s < nsub run the guard of sub-step s.
__global__ void __launch_bounds__(kBlock) k_halo_unpack_nbr(int W, int halo, int rows_lo, int rows_hi, long hi_off,
                                                            const double* __restrict__ recv, int ws, int rank,
                                                            double radius, int nsub, double2* __restrict__ wpos,
                                                            int32_t* __restrict__ flag) {
    const long t = (long)blockIdx.x * kBlock + threadIdx.x;
    const long nlo = (long)rows_lo * W, nhi = (long)rows_hi * W, rs = (long)halo * W, r8 = 8l * nsub;
    if (t < nlo) {
        const double2* src = reinterpret_cast<const double2*>(recv + nbr_chunk_off(rank - 1, rank, ws, r8, 2 * rs) + r8);
        wpos[t] = src[rs - nlo + t];
    } else if (t < nlo + nhi) {
        const double2* src = reinterpret_cast<const double2*>(recv + nbr_chunk_off(rank + 1, rank, ws, r8, 2 * rs) + r8);
        wpos[hi_off + (t - nlo)] = src[t - nlo];
    }
    if (blockIdx.x == 0 && threadIdx.x < nsub && !halo_guard_ok_nbr(recv, threadIdx.x, ws, rank, r8, 2 * rs, radius))
        atomicOr(flag, 1);
}

}  // namespace

extern "C" int64_t cbf_halo_nbr_elems(int32_t W, int32_t halo, int32_t nsub, int32_t world_size, int32_t rank) {
    if (W <= 0 || halo <= 0 || nsub < 1 || world_size < 1 || rank < 0 || rank >= world_size) return -1;
    const long r8 = 8l * nsub, rs2 = 2l * halo * W;
    return (int64_t)(world_size * r8 + (rank > 0 ? rs2 : 0) + (rank + 1 < world_size ? rs2 : 0));
}

extern "C" int cbf_halo_pack_nbr(int32_t W, int32_t halo, int64_t n_own, const double* own, uint64_t* ext_keys,
                                 int32_t nsub, int32_t world_size, int32_t rank, double* send, void* stream) {
    if (W <= 0 || halo <= 0 || n_own < 2l * halo * W || !own || !ext_keys || !send || nsub < 1 || nsub > 64 ||
        world_size < 1 || rank < 0 || rank >= world_size)
        return CBF_EINVAL;
    const long rs = (long)halo * W;
    const long n = (rank > 0 ? rs : 0) + (rank + 1 < world_size ? rs : 0);
    hipLaunchKernelGGL(k_halo_pack_nbr, dim3(nblk(n > 0 ? n : 1)), dim3(kBlock), 0, (hipStream_t)stream, W, halo,
                       (long)n_own, reinterpret_cast<const double2*>(own),
                       reinterpret_cast<unsigned long long*>(ext_keys), nsub, world_size, rank, send);
    return (int)hipGetLastError();
}

extern "C" int cbf_halo_unpack_nbr(int32_t W, int32_t halo, int32_t rows_lo, int32_t rows_hi, int64_t hi_row_offset,
                                   const double* recv, int32_t world_size, int32_t rank, double radius, int32_t nsub,
                                   double* wpos, int32_t* flag, void* stream) {
    if (W <= 0 || halo <= 0 || rows_lo < 0 || rows_hi < 0 || rows_lo > halo || rows_hi > halo || !recv || !wpos ||
        !flag || world_size < 1 || rank < 0 || rank >= world_size || nsub < 1 || nsub > 64 ||
        (rows_lo > 0 && rank == 0) || (rows_hi > 0 && rank == world_size - 1) || hi_row_offset < 0)
        return CBF_EINVAL;
    const long n = (long)(rows_lo + rows_hi) * W;
    hipLaunchKernelGGL(k_halo_unpack_nbr, dim3(nblk(n > 0 ? n : 1)), dim3(kBlock), 0, (hipStream_t)stream, W, halo,
                       rows_lo, rows_hi, (long)hi_row_offset * W, recv, world_size, rank, radius, nsub,
                       reinterpret_cast<double2*>(wpos), flag);
    return (int)hipGetLastError();
}

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
