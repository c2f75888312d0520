// lattice.hpp -- helpers shared by the lattice-step filters (swarm.hip: reference barrier,
// hocbf.hip: Euclidean HOCBF mode): halo-guard extents and argument checks.
#pragma once

#include "cbf_device.hpp"
#include "cells.hpp"

namespace cbf {

// CBF_XCD_REMAP: blocks are dealt round-robin over the 8 XCDs (b and b+8 share one L2), so
// consecutive blocks -- which read the same cell rows of the sorted arrays -- would pull the same
// lines into every XCD's L2.  The remap is a bijection of [0, nb) that hands each XCD one
// contiguous range of logical blocks.  Speed only: placement is never assumed for correctness.
#ifndef CBF_XCD_REMAP
#define CBF_XCD_REMAP 1
#endif

__device__ __forceinline__ int xcd_block() {
#if CBF_XCD_REMAP
    const int b = blockIdx.x, nb = gridDim.x;
    const int q = nb >> 3, rem = nb & 7, x = b & 7, j = b >> 3;
    return (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + j;
#else
    return blockIdx.x;
#endif
}

__device__ __forceinline__ int wave_min_i(int v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ int wave_max_i(int v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

__device__ __forceinline__ double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = pmin(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = pmax(v, __shfl_xor(v, o, 64));
    return v;
}

// Per-wave extents of the new owned y (halo guard of the sharded step): {min, max, max over rows
// < row_end - guard, min over rows >= row_begin + guard}; lane 0 writes part[4 * wave].  Per wave,
// not per block: a block-wide barrier at the end would hold every wave of a block until its
// slowest finished.
__device__ __forceinline__ void wave_extents(double e0, double e1, double e2, double e3, double* part, long wave) {
    const double m0 = wave_min(e0), m1 = wave_max(e1), m2 = wave_max(e2), m3 = wave_min(e3);
    if ((threadIdx.x & 63) == 0) {
        double* o = part + 4 * wave;
        o[0] = m0;
        o[1] = m1;
        o[2] = m2;
        o[3] = m3;
    }
}

__device__ __forceinline__ void ext_accumulate(int r, int row_begin, int row_end, int guard_rows, double ny,
                                               double& e0, double& e1, double& e2, double& e3) {
    e0 = pmin(e0, ny);
    e1 = pmax(e1, ny);
    if (r < row_end - guard_rows) e2 = pmax(e2, ny);
    if (r >= row_begin + guard_rows) e3 = pmin(e3, ny);
}

// The row tests of the reference-barrier lattice filter as bounds on the window index
// w = (r - win_row0) W + c (0 <= c < W): r < X <=> w < (X - win_row0) W and r >= Y <=>
// w >= (Y - win_row0) W, so the kernels never divide by W.
struct WinBounds {
    int own_lo, own_hi;  // owned rows [row_begin, row_end); output index k = w - own_lo
    int cnt_lo, cnt_hi;  // rows whose solves are counted
    int g_hi;            // rows < row_end - guard_rows (halo-guard extents)
    int g_lo;            // rows >= row_begin + guard_rows
};
inline int win_bound(long row, int win_row0, int W, long nwin) {
    const long v = (row - win_row0) * (long)W;  // clamped to [-1, nwin + 1]: same answers for w in [0, nwin)
    return (int)(v < -1 ? -1 : (v > nwin + 1 ? nwin + 1 : v));
}
inline WinBounds make_win_bounds(int W, int win_row0, long nwin, int row_begin, int row_end, int cnt_begin,
                                 int cnt_end, int guard_rows) {
    WinBounds B;
    B.own_lo = win_bound(row_begin, win_row0, W, nwin);
    B.own_hi = win_bound(row_end, win_row0, W, nwin);
    B.cnt_lo = win_bound(cnt_begin, win_row0, W, nwin);
    B.cnt_hi = win_bound(cnt_end, win_row0, W, nwin);
    B.g_hi = win_bound((long)row_end - guard_rows, win_row0, W, nwin);
    B.g_lo = win_bound((long)row_begin + guard_rows, win_row0, W, nwin);
    return B;
}
// ext_accumulate for an owned agent given by its window index
__device__ __forceinline__ void ext_accumulate_w(int w, const WinBounds& B, double ny, double& e0, double& e1,
                                                 double& e2, double& e3) {
    e0 = pmin(e0, ny);
    e1 = pmax(e1, ny);
    if (w < B.g_hi) e2 = pmax(e2, ny);
    if (w >= B.g_lo) e3 = pmin(e3, ny);
}

// Cell of a position (the bin kernels' formula).
__device__ __forceinline__ int cell_of(const CellGrid& G, double x, double y) {
    return cell_coord(y, G.y0, G.inv_h, G.ny) * G.nx + cell_coord(x, G.x0, G.inv_h, G.nx);
}

// Counting-sort binning of one agent per lane (cell < 0: none): the lane's rank in its cell.
// Consecutive lanes of equal cell form a run served by one atomic (the agents arrive in the
// previous cell order, so runs are long).  Every lane of the wave must call it.
__device__ __forceinline__ int run_rank(int cell, int32_t* __restrict__ count) {
    const int lane = threadIdx.x & 63;
    const int cprev = __shfl_up(cell, 1, 64);
    const bool leader = lane == 0 || cell != cprev;
    const unsigned long long lm = __ballot(leader);
    const unsigned long long upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const int my_leader = 63 - __clzll(lm & upto);
    const unsigned long long above = lm & ~upto;
    const int next = above ? __ffsll((long long)above) - 1 : 64;
    int base = 0;
    if (leader && cell >= 0) base = atomicAdd(&count[cell], next - lane);
    base = __shfl(base, my_leader, 64);
    return base + lane - my_leader;
}

// This lane's record index in the queue area (sub-queue q at [q qcap, (q + 1) qcap), length at
// hardq[32 (1 + q)]); every active lane of the wave that calls it appends one entry, with one
// atomic per wave.  The capacity is sized for kBlock-lane filter blocks sharing a sub-queue; a
// larger block (the window tile's 512 egos) can find its sub-queue full, and its remaining lanes
// then take the next sub-queues (the counter of a full one runs past qcap: the queue kernels read
// min(length, qcap)).  The sub-queues together hold every agent, so a slot is always found.
__device__ __forceinline__ long subq_append(int32_t* hardq, int q, long qcap) {
    const int lane = threadIdx.x & 63;
    long rec = -1;
    bool need = true;
    for (int t = 0; t < kSubQ; ++t) {
        const unsigned long long m = __ballot(need);
        if (!m) break;
        const int qq = (q + t) & (kSubQ - 1);
        const int leader = __ffsll((long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(&hardq[32 * (1 + qq)], __popcll(m));
        base = __shfl(base, leader, 64);
        if (need) {
            const long sl = base + __popcll(m & ((1ull << lane) - 1ull));
            if (sl < qcap) {
                rec = (long)qq * qcap + sl;
                need = false;
            }
        }
    }
    return rec;
}

// The queue kernels: 64-lane blocks, block g serving sub-queue g % kSubQ as its (g / kSubQ)-th of
// per_q blocks.  Of a sub-queue of length nq, nwork = min(per_q, ceil(nq / 64)) blocks work, lane
// i of the k-th taking entries k 64 + i, then + nwork 64, ...; visit(entry) per entry.  The working
// blocks of a sub-queue count themselves done as soon as they have read the length (a block needs
// only the length: the records stay untouched until the next advance), so the counter's return
// trip overlaps the solves instead of ending the kernel; the last one to count empties the
// sub-queue (length and done counter) at its end, so the next advance starts from empty queues
// with no extra launch.  No fence: a block is one wave whose load of the length has returned
// before lane 0's atomic, and nothing the reset races with is written by the queue kernels.  A
// block k >= nwork that reads the length after the reset sees 0 and is still idle (any smaller
// length gives it no work either); a working block cannot read it after the reset, which needs
// its own count first.
template <class Visit>
__device__ __forceinline__ void drain_subq(int32_t* __restrict__ hardq, int per_q, long qcap, Visit&& visit) {
    const int q = blockIdx.x % kSubQ, k = blockIdx.x / kSubQ;
    const int nq0 = hardq[32 * (1 + q)];
    const int nq = nq0 < qcap ? nq0 : (int)qcap;  // (a full sub-queue's counter runs past qcap: subq_append)
    const int need = (nq + 63) / 64;
    const int nwork = need < per_q ? need : per_q;
    if (k >= nwork) return;
    int done = 0;
    if (threadIdx.x == 0) done = atomicAdd(&hardq[32 * (1 + kSubQ + q)], 1);
    for (int i = k * 64 + threadIdx.x; i < nq; i += nwork * 64) visit(q, i);
    if (threadIdx.x == 0 && done == nwork - 1) {
        hardq[32 * (1 + q)] = 0;
        hardq[32 * (1 + kSubQ + q)] = 0;
    }
}

// Rollout statistics of the lattice step (`stats`, device uint64[1024] = 64 slots of 16 words,
// one 128-B line each; a wave adds into slot (its index & 63), the host sums or maxes over the
// slots).  Counted over the egos of the counted rows.  The two violations are the bits of
// non-negative doubles (monotone as uint64, so atomicMax is an exact maximum); the smallest
// neighbour distance^2 is kept as kDistKeyTop - bits(s) under atomicMax, so a zero-filled array
// reads as "no neighbour pair".  Word layout: cbf_amd.h (CBF_STAT_*).
constexpr unsigned long long kDistKeyTop = 0x7FF0000000000000ull;
// Slots 0..62 take the atomics; slot 63 only ever holds a copy of the three maxima taken at the
// end of an earlier step (stat_snapshot), read by the filter waves to skip lanes that cannot
// raise them.  Zeroing the array zeroes the copy too, so the skip stays exact across resets.
constexpr int kStatSlots = 63, kStatSnap = 63;
__device__ __forceinline__ long stat_slot(long i) { return i % kStatSlots; }

__device__ __forceinline__ unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }

}  // namespace cbf
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_max_u32(unsigned int);
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_min_u32(unsigned int);
namespace cbf {

// Wave-wide max / min of 64-bit keys as two 32-bit DPP reductions (high words, then the low words
// of the lanes holding the extreme high word): about half the instructions of a 64-bit shuffle
// tree.  Every lane of the wave must call them; all lanes get the result.
__device__ __forceinline__ unsigned long long wave_umax64(unsigned long long v) {
    const unsigned hi = (unsigned)(v >> 32);
    const unsigned mh = __ockl_wfred_max_u32(hi);
    const unsigned ml = __ockl_wfred_max_u32(hi == mh ? (unsigned)v : 0u);
    return ((unsigned long long)mh << 32) | ml;
}
__device__ __forceinline__ unsigned long long wave_umin64(unsigned long long v) {
    const unsigned hi = (unsigned)(v >> 32);
    const unsigned mh = __ockl_wfred_min_u32(hi);
    const unsigned ml = __ockl_wfred_min_u32(hi == mh ? (unsigned)v : 0xFFFFFFFFu);
    return ((unsigned long long)mh << 32) | ml;
}

// One wave's contribution.  solved: an agent-QP ran for this lane's ego (>= 1 neighbour);
// seidel: its QP went to the full solve (queued); fin: its status code is final here (code,
// viol = violation of the solved rows, vorig = violation of the original rows); d2: smallest
// neighbour distance^2 of the ego (+inf if none).  Every lane of the wave must call it.  The
// maxima and the minimum are taken over the bits of the non-negative doubles (only values > 0 enter
// the maxima), which order like the values.
__device__ __forceinline__ void wave_stats(unsigned long long* __restrict__ st, long wave, bool solved, bool seidel,
                                           bool fin, int code, bool binding, double viol, double vorig, double d2) {
    const bool opt = fin && code == CBF_STATUS_OPTIMAL, rel = fin && code == CBF_STATUS_RELAXED;
    const bool inf = fin && (code == CBF_STATUS_BOX_INFEASIBLE || code == CBF_STATUS_RELAX_CAP);
    const unsigned long long m_sol = __ballot(solved), m_sei = __ballot(seidel), m_opt = __ballot(opt),
                             m_rel = __ballot(rel), m_inf = __ballot(inf), m_bnd = __ballot(fin && binding);
    // only values beyond the snapshot (a maximum already recorded) can change the result
    const unsigned long long* snap = st + 16 * kStatSnap;
    const bool po = opt && viol > 0.0 && dbits(viol) > snap[CBF_STAT_VIOL_OPTIMAL];
    const bool pr = rel && vorig > 0.0 && dbits(vorig) > snap[CBF_STAT_VIOL_ORIGINAL];
    const bool pd = d2 < INFINITY && kDistKeyTop - dbits(d2) > snap[CBF_STAT_MIN_DIST2];
    unsigned long long vo = 0, vr = 0, dm = 0;
    if (__ballot(po)) vo = wave_umax64(po ? dbits(viol) : 0ull);
    if (__ballot(pr)) vr = wave_umax64(pr ? dbits(vorig) : 0ull);
    if (__ballot(pd)) dm = kDistKeyTop - wave_umin64(pd ? dbits(d2) : kDistKeyTop);
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* s = st + 16 * stat_slot(wave);
        if (m_sol) atomicAdd(&s[CBF_STAT_SOLVES], (unsigned long long)__popcll(m_sol));
        if (m_opt) atomicAdd(&s[CBF_STAT_OPTIMAL], (unsigned long long)__popcll(m_opt));
        if (m_rel) atomicAdd(&s[CBF_STAT_RELAXED], (unsigned long long)__popcll(m_rel));
        if (m_inf) atomicAdd(&s[CBF_STAT_INFEASIBLE], (unsigned long long)__popcll(m_inf));
        if (m_sei) atomicAdd(&s[CBF_STAT_SEIDEL], (unsigned long long)__popcll(m_sei));
        if (m_bnd) atomicAdd(&s[CBF_STAT_BINDING], (unsigned long long)__popcll(m_bnd));
        if (vo) atomicMax(&s[CBF_STAT_VIOL_OPTIMAL], vo);
        if (vr) atomicMax(&s[CBF_STAT_VIOL_ORIGINAL], vr);
        if (dm) atomicMax(&s[CBF_STAT_MIN_DIST2], dm);
    }
}

// The lattice filters' path when the build is flagged unusable: window agent slot (identity order,
// the cell-sorted copies are not read) reports CBF_STATUS_WORKSPACE_ERROR for an owned agent, with
// u = 0 and no neighbours; positions are left as they are; the step counts as one error, and the
// cell order the build recorded (hardq[2..7]) is dropped.
__device__ __forceinline__ void lattice_error_tail(int W, int row_begin, int row_end, int win_row0, long nwin,
                                                   long slot, double2* __restrict__ u, int32_t* __restrict__ status,
                                                   int32_t* __restrict__ cnt, unsigned long long* __restrict__ stats,
                                                   double* __restrict__ ext_part, long wave,
                                                   int32_t* __restrict__ hardq) {
    // the sorted copies of this build are not a permutation: the next build walks identity order
    if (slot == 0) hardq[2] = 0;
    if (slot < nwin) {
        const int r = win_row0 + (int)(slot / W), c = (int)(slot % W);
        if (r >= row_begin && r < row_end) {
            // u / status / cnt are null in the inner timesteps of a run or an exchange cycle
            const long k = (long)(r - row_begin) * W + c;
            if (u) u[k] = make_double2(0.0, 0.0);
            if (status) status[k] = CBF_STATUS_WORKSPACE_ERROR;
            if (cnt) cnt[k] = 0;
        }
    }
    if (stats && slot == 0) atomicAdd(&stats[CBF_STAT_ERRORS], 1ull);
    if (ext_part && (threadIdx.x & 63) == 0) {
        double* o = ext_part + 4 * wave;
        o[0] = INFINITY;
        o[1] = -INFINITY;
        o[2] = -INFINITY;
        o[3] = INFINITY;
    }
}

// Per-lane status counts and violation maxima of a queue kernel, summed over the wave (every lane
// of the wave must call it, after its loop).
__device__ __forceinline__ void wave_stats_counts(unsigned long long* __restrict__ st, long wave, int n_opt, int n_rel,
                                                  int n_inf, int n_bnd, int n_sei, double vo, double vr) {
    for (int o = 32; o > 0; o >>= 1) {
        n_sei += __shfl_xor(n_sei, o, 64);
        n_opt += __shfl_xor(n_opt, o, 64);
        n_rel += __shfl_xor(n_rel, o, 64);
        n_inf += __shfl_xor(n_inf, o, 64);
        n_bnd += __shfl_xor(n_bnd, o, 64);
    }
    vo = wave_max(vo);
    vr = wave_max(vr);
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* s = st + 16 * stat_slot(wave);
        if (n_opt) atomicAdd(&s[CBF_STAT_OPTIMAL], (unsigned long long)n_opt);
        if (n_rel) atomicAdd(&s[CBF_STAT_RELAXED], (unsigned long long)n_rel);
        if (n_inf) atomicAdd(&s[CBF_STAT_INFEASIBLE], (unsigned long long)n_inf);
        if (n_bnd) atomicAdd(&s[CBF_STAT_BINDING], (unsigned long long)n_bnd);
        if (n_sei) atomicAdd(&s[CBF_STAT_SEIDEL], (unsigned long long)n_sei);
        if (vo > 0.0) atomicMax(&s[CBF_STAT_VIOL_OPTIMAL], dbits(vo));
        if (vr > 0.0) atomicMax(&s[CBF_STAT_VIOL_ORIGINAL], dbits(vr));
    }
}

// Refresh the snapshot slot: the maxima over slots 0..62 (and the old copy) into slot 63, by one
// 64-lane block.  Values read mid-update are earlier ones, which are still valid lower bounds.
__device__ __forceinline__ void stat_snapshot(unsigned long long* __restrict__ st) {
    const int l = threadIdx.x;
    unsigned long long a = 0, b = 0, c = 0;
    if (l <= kStatSlots) {  // lane 63 reads the old copy
        a = st[16 * l + CBF_STAT_VIOL_OPTIMAL];
        b = st[16 * l + CBF_STAT_VIOL_ORIGINAL];
        c = st[16 * l + CBF_STAT_MIN_DIST2];
    }
    a = wave_umax64(a);
    b = wave_umax64(b);
    c = wave_umax64(c);
    if (l == 0) {
        unsigned long long* s = st + 16 * kStatSnap;
        s[CBF_STAT_VIOL_OPTIMAL] = a;
        s[CBF_STAT_VIOL_ORIGINAL] = b;
        s[CBF_STAT_MIN_DIST2] = c;
    }
}

// Reduces nparts per-wave extents to out[4] (one-block kernel, defined in swarm.hip).
void launch_extents_finalize(int nparts, const double* part, double* out, hipStream_t s);

// partial extents: one record per wave of the filter grid, then one per hard-QP block
inline long lattice_ext_waves(long win_n) { return (win_n + kBlock - 1) / kBlock * (kBlock / 64); }
// the HOCBF wide kernel: one queued ego per 64-lane block at a time, kWidePerQ blocks per
// sub-queue (~10 k queued egos at cfg4, ~160 per sub-queue: one ego per block; 64 blocks per
// sub-queue: HOCBF step 204.8 against 202.8 us)
#ifndef CBF_WIDE_PER_Q
#define CBF_WIDE_PER_Q 256
#endif
constexpr int kWidePerQ = CBF_WIDE_PER_Q;
inline int lattice_wide_blocks(long) { return kSubQ * kWidePerQ; }
// the hard-QP kernel of the lattice step: kHardPerQ 64-lane blocks per sub-queue (2048 lanes: the
// ~4.6 k entries per sub-queue at cfg4f in ~2 passes, the ~50 at cfg4 in one block)
#ifndef CBF_HARD_PER_Q
#define CBF_HARD_PER_Q 32
#endif
constexpr int kHardPerQ = CBF_HARD_PER_Q;
inline int lattice_hard_blocks(long) { return kSubQ * kHardPerQ; }
// (the HOCBF step has both: its hard kernel's blocks -- up to 128 per sub-queue -- then the wide
// kernel's)
inline size_t lattice_ext_bytes(long win_n) {
    const long hb = lattice_hard_blocks(win_n), wb = lattice_wide_blocks(win_n), hh = kSubQ * 128l;
    return align256(32 * (size_t)(lattice_ext_waves(win_n) + (hb > hh ? hb : hh) + wb));
}

inline int check_lattice(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                         int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, void* workspace,
                         size_t workspace_bytes) {
    if (!p || !grid || W <= 0 || H <= 0) return CBF_EINVAL;
    if (row_begin < 0 || row_end > H || row_begin >= row_end) return CBF_EINVAL;
    if (win_row0 < 0 || win_rows <= 0 || win_row0 + win_rows > H) return CBF_EINVAL;
    // owned rows plus one neighbour row on each side (where it exists) must be in the window
    if (win_row0 > (row_begin > 0 ? row_begin - 1 : 0)) return CBF_EINVAL;
    if (win_row0 + win_rows < (row_end < H ? row_end + 1 : H)) return CBF_EINVAL;
    if ((long)W * win_rows >= (1l << 28)) return CBF_EINVAL;  // 32-bit byte offsets into the sorted copies (ld_slot)
    if (!pos || !workspace) return CBF_EINVAL;
    if (grid->nx <= 0 || grid->ny <= 0 || !(grid->inv_h > 0) || !(1.0 / grid->inv_h >= sqrt(p->cull_t)))
        return CBF_EINVAL;
    if ((long)grid->nx * grid->ny > (1l << 30)) return CBF_EINVAL;
    if (workspace_bytes < cbf_lattice_workspace_size(W, win_rows, grid)) return CBF_EINVAL;
    return 0;
}

}  // namespace cbf
