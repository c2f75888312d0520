// cells.hip -- cell-list construction kernels (counting sort by uniform-grid cell).
#include "cbf_device.hpp"
#include "cells.hpp"

namespace cbf {
namespace {

__global__ void __launch_bounds__(kBlock) k_bin(CellGrid G, int n, const double2* __restrict__ pos,
                                                int32_t* __restrict__ count, int2* __restrict__ cs) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double2 p = pos[i];
    const int c = cell_coord(p.y, G.y0, G.inv_h, G.ny) * G.nx + cell_coord(p.x, G.x0, G.inv_h, G.nx);
    const int slot = atomicAdd(&count[c], 1);
    cs[i] = make_int2(c, slot);
}

__device__ __forceinline__ int block_sum(int v, int* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    int t = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kBlock / 64; ++w) t += red[w];
    return t;  // valid in thread 0
}

__global__ void __launch_bounds__(kBlock) k_tile_reduce(const int32_t* __restrict__ count, long ncell,
                                                        int32_t* __restrict__ tilesum) {
    __shared__ int red[kBlock / 64];
    const long base = (long)blockIdx.x * kScanTile + threadIdx.x * 8;
    int v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (base + k < ncell) v += count[base + k];
    const int t = block_sum(v, red);
    if (threadIdx.x == 0) tilesum[blockIdx.x] = t;
}

// Exclusive scan: each tile adds the sum of all previous tiles (summed redundantly per block:
// a few hundred ints) to its own block-local scan.
__global__ void __launch_bounds__(kBlock) k_tile_scan(int32_t* __restrict__ count, long ncell,
                                                      const int32_t* __restrict__ tilesum,
                                                      int32_t* __restrict__ start) {
    __shared__ int red[kBlock / 64];
    __shared__ int wtot[kBlock / 64];
    __shared__ int s_off;
    int v = 0;
    for (int t = threadIdx.x; t < (int)blockIdx.x; t += kBlock) v += tilesum[t];
    const int off = block_sum(v, red);
    if (threadIdx.x == 0) s_off = off;
    const long base = (long)blockIdx.x * kScanTile + threadIdx.x * 8;
    int c[8];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c[k] = (base + k < ncell) ? count[base + k] : 0;
        tot += c[k];
    }
    // leave the counts zeroed for the next build (no memset node needed in a captured step)
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (base + k < ncell) count[base + k] = 0;
    // inclusive wave scan of thread totals
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wtot[wid] = inc;
    __syncthreads();
    int wpre = 0;
    for (int w = 0; w < wid; ++w) wpre += wtot[w];
    int run = s_off + wpre + inc - tot;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (base + k < ncell) start[base + k] = run;
        run += c[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) start[ncell] = run;
}

__global__ void __launch_bounds__(kBlock) k_scatter(int n, const int2* __restrict__ cs,
                                                    const int32_t* __restrict__ start,
                                                    const double2* __restrict__ pos, const double2* __restrict__ vel,
                                                    double2* __restrict__ spos, double2* __restrict__ svel,
                                                    int32_t* __restrict__ sidx) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int2 c = cs[i];
    if (c.x < 0) return;
    const int d = start[c.x] + c.y;
    spos[d] = pos[i];
    svel[d] = vel[i];
    sidx[d] = i;
}

inline int nblk(long n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

void launch_scan(const CellWs& W, hipStream_t s) {
    hipLaunchKernelGGL(k_tile_reduce, dim3(W.ntiles), dim3(kBlock), 0, s, W.count, W.ncell, W.tilesum);
    hipLaunchKernelGGL(k_tile_scan, dim3(W.ntiles), dim3(kBlock), 0, s, W.count, W.ncell, W.tilesum, W.start);
}

int scan_and_scatter(const CellGrid& G, const CellWs& W, int n, const double2* pos, const double2* vel,
                     hipStream_t s) {
    launch_scan(W, s);
    hipLaunchKernelGGL(k_scatter, dim3(nblk(n)), dim3(kBlock), 0, s, n, W.cs, W.start, pos, vel, W.spos, W.svel,
                       W.sidx);
    return (int)hipGetLastError();
}

int build_cells(const CellGrid& G, const CellWs& W, int n, const double2* pos, const double2* vel, const int32_t*,
                hipStream_t s) {
    hipLaunchKernelGGL(k_bin, dim3(nblk(n)), dim3(kBlock), 0, s, G, n, pos, W.count, W.cs);
    return scan_and_scatter(G, W, n, pos, vel, s);
}

}  // namespace cbf
