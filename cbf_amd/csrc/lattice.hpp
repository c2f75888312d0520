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

// End of a 64-lane queue kernel (every block has read hardq[0]): the last block to finish
// empties the queue, so an advance run again without a build starts from an empty queue.  No
// fence: the block is one wave whose load of hardq[0] has returned (the loop used it) before
// lane 0's atomic, and nothing the reset could race with is written by the queue kernels.
__device__ __forceinline__ void hard_queue_done(int32_t* hardq) {
    if (threadIdx.x == 0) {
        if (atomicAdd(&hardq[1], 1) == (int)gridDim.x - 1) {
            hardq[0] = 0;
            hardq[1] = 0;
        }
    }
}

// Reduces nparts per-wave extents to out[4] (one-block kernel, defined in swarm.hip).
void launch_extents_finalize(int nparts, const double* part, double* out, hipStream_t s);

// partial extents: one record per wave of the filter grid, then one per hard-QP block
inline long lattice_ext_waves(long win_n) { return (win_n + kBlock - 1) / kBlock * (kBlock / 64); }
// grid of the HOCBF wide kernel (64-lane blocks): 256 x 64 lanes cover the ~10 k queued egos of
// cfg4 one per lane; every block ends with one atomic on the done counter, so a larger grid only
// lengthens that serialised chain (1024 blocks: advance 231 vs 221 us, tools/ablate.py set wide)
#ifndef CBF_WIDE_BLOCKS
#define CBF_WIDE_BLOCKS 256
#endif
constexpr int kWideBlocks = CBF_WIDE_BLOCKS;
constexpr int kQueueBlocksMax = kHardBlocks > kWideBlocks ? kHardBlocks : kWideBlocks;
inline size_t lattice_ext_bytes(long win_n) {
    return align256(32 * (size_t)(lattice_ext_waves(win_n) + kQueueBlocksMax));
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
    if ((long)W * win_rows >= (1l << 31)) return CBF_EINVAL;
    if (!pos || !workspace) return CBF_EINVAL;
    if (grid->nx <= 0 || grid->ny <= 0 || !(grid->inv_h > 0) || !(1.0 / grid->inv_h >= sqrt(p->cull_t)))
        return CBF_EINVAL;
    if ((long)grid->nx * grid->ny > (1l << 30)) return CBF_EINVAL;
    if (workspace_bytes < cbf_lattice_workspace_size(W, win_rows, grid)) return CBF_EINVAL;
    return 0;
}

}  // namespace cbf
