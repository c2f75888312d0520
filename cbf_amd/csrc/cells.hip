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

// Single-pass exclusive scan of the cell counts (decoupled look-back).  Tiles are taken in
// ticket order, so a tile only waits on tiles whose blocks are already running.  Tile status is
// one 64-bit word {epoch:30 | flag:2 | value:32} written and read with agent-scope relaxed
// atomics (the payload travels inside the flag word, so no fence is needed); the epoch (bumped
// by the last tile) makes words of earlier launches invisible without any reset pass.  The
// kernel re-zeroes the counts it consumed.  Spins are bounded; a timeout sets sctl[2].
constexpr unsigned long long kFlagAgg = 1ull << 32, kFlagInc = 2ull << 32;

__device__ __forceinline__ unsigned long long ld_state(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_state(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kBlock) k_scan_onepass(int32_t* __restrict__ count, long ncell, int ntiles,
                                                         int32_t* __restrict__ start,
                                                         unsigned long long* __restrict__ tstate,
                                                         int32_t* __restrict__ sctl) {
    __shared__ int s_tile, s_excl;
    __shared__ unsigned s_epoch;
    __shared__ int wtot[kBlock / 64];
    if (threadIdx.x == 0) {
        s_tile = atomicAdd(&sctl[0], 1);
        s_epoch = (unsigned)__hip_atomic_load(&sctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int tile = s_tile;
    const unsigned long long ep = (unsigned long long)(s_epoch & 0x3FFFFFFFu) << 34;
    const long base = (long)tile * kScanTile + threadIdx.x * 8;
    int c[8];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c[k] = (base + k < ncell) ? count[base + k] : 0;
        tot += c[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (base + k < ncell) count[base + k] = 0;  // leave the counts zeroed for the next build
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wtot[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        int agg = 0;
        for (int w = 0; w < kBlock / 64; ++w) agg += wtot[w];
        int excl = 0;
        if (tile == 0) {
            st_state(&tstate[0], ep | kFlagInc | (unsigned)agg);
        } else {
            st_state(&tstate[tile], ep | kFlagAgg | (unsigned)agg);
            int j = tile - 1;
            long spins = 0;
            while (j >= 0) {
                const unsigned long long v = ld_state(&tstate[j]);
                const bool mine = (v & ~((1ull << 34) - 1)) == ep;
                const unsigned long long fl = v & (3ull << 32);
                if (mine && fl != 0) {
                    excl += (int)(unsigned)(v & 0xFFFFFFFFull);
                    if (fl == kFlagInc) break;
                    --j;
                } else if (++spins > (1l << 26)) {
                    sctl[2] = 1;
                    break;
                } else {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            st_state(&tstate[tile], ep | kFlagInc | (unsigned)(excl + agg));
        }
        s_excl = excl;
        if (tile == ntiles - 1) {  // last ticket: every other block has read the epoch already
            start[ncell] = excl + agg;
            sctl[0] = 0;
            __hip_atomic_store(&sctl[1], (int)((s_epoch + 1) & 0x3FFFFFFFu), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    int wpre = 0;
    for (int w = 0; w < wid; ++w) wpre += wtot[w];
    int run = s_excl + wpre + inc - tot;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (base + k < ncell) start[base + k] = run;
        run += c[k];
    }
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
    hipLaunchKernelGGL(k_scan_onepass, dim3(W.ntiles), dim3(kBlock), 0, s, W.count, W.ncell, W.ntiles, W.start, W.tstate,
                       W.sctl);
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
