// cells.hip -- cell-list construction kernels (counting sort by uniform-grid cell).
#include "cbf_device.hpp"
#include "cells.hpp"

namespace cbf {
namespace {

__global__ void __launch_bounds__(kBlock) k_bin(CellGrid G, int n, const double2* __restrict__ pos,
                                                int32_t* __restrict__ count, int2* __restrict__ cs,
                                                int32_t* __restrict__ sctl) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) build_begin(sctl, n, (long)G.nx * G.ny);
    if (i >= n) return;
    const double2 p = pos[i];
    const int c = cell_coord(p.y, G.y0, G.inv_h, G.ny) * G.nx + cell_coord(p.x, G.x0, G.inv_h, G.nx);
    const int slot = atomicAdd(&count[c], 1);
    cs[i] = make_int2(c, slot);
}

// Single-pass exclusive scan of the cell counts (decoupled look-back).  Tile = block index: the
// dispatcher hands out workgroups in increasing order, so a tile only waits on tiles whose blocks
// are already resident.  Tile status is one 64-bit word {epoch:30 | flag:2 | value:32} written
// and read with agent-scope relaxed atomics (the payload travels inside the flag word, so no
// fence is needed); the epoch (advanced before each scan by the bin kernel) makes words of
// earlier launches invisible without a reset pass.  The epoch load and the count loads are
// independent, so the critical path is load -> publish/look-back -> store.  The kernel re-zeroes
// the counts it consumed.  Spins are bounded: a look-back that gives up sets sctl[2], which the
// filter kernels turn into CBF_STATUS_WORKSPACE_ERROR for every ego of that step (the cell starts
// are then wrong); the next bin kernel clears it (build_begin).  CBF_SCAN_TEST_TIMEOUT = 1 (a test build only)
// makes every look-back give up at once, so the reporting path can be tested deterministically.
constexpr unsigned long long kFlagAgg = 1ull << 32, kFlagInc = 2ull << 32;
#ifndef CBF_SCAN_SPIN_LIMIT
#define CBF_SCAN_SPIN_LIMIT (1l << 24)
#endif
#ifndef CBF_SCAN_TEST_TIMEOUT
#define CBF_SCAN_TEST_TIMEOUT 0
#endif

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
    __shared__ int s_excl;
    __shared__ int wtot[kBlock / 64];
    const int tile = blockIdx.x;
    const unsigned epoch = (unsigned)__hip_atomic_load(&sctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long ep = (unsigned long long)(epoch & 0x3FFFFFFFu) << 34;
    constexpr int kPer = kScanTile / kBlock;  // cells per lane, a multiple of 4
    const long base = (long)tile * kScanTile + threadIdx.x * kPer;
    int c[kPer];
    int tot = 0;
    if (base + kPer <= ncell) {  // 16-B loads (base is a multiple of kPer ints)
#pragma unroll
        for (int v = 0; v < kPer / 4; ++v) {
            const int4 a = *reinterpret_cast<const int4*>(count + base + 4 * v);
            c[4 * v] = a.x, c[4 * v + 1] = a.y, c[4 * v + 2] = a.z, c[4 * v + 3] = a.w;
            *reinterpret_cast<int4*>(count + base + 4 * v) = make_int4(0, 0, 0, 0);  // zeroed for the next build
        }
    } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            c[k] = (base + k < ncell) ? count[base + k] : 0;
            if (base + k < ncell) count[base + k] = 0;
        }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) tot += c[k];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wtot[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        // wave-parallel look-back: lane l reads the status of tile (top - l), 64 predecessors per
        // round trip; the window is summed down to its nearest inclusive entry
        int agg = 0;
        for (int w = 0; w < kBlock / 64; ++w) agg += wtot[w];
        int excl = 0;
        if (tile == 0) {
            if (lane == 0) st_state(&tstate[0], ep | kFlagInc | (unsigned)agg);
        } else {
            if (lane == 0) st_state(&tstate[tile], ep | kFlagAgg | (unsigned)agg);
            int top = tile - 1;
            long spins = 0;
            while (true) {
                const int idx = top - lane;
                const unsigned long long v = idx >= 0 ? ld_state(&tstate[idx]) : (ep | kFlagInc);
                const bool ready = (v & ~((1ull << 34) - 1)) == ep && (v & (3ull << 32)) != 0;
                const bool incl = ready && (v & (3ull << 32)) == kFlagInc;
                const unsigned long long im = __ballot(incl), nr = __ballot(!ready);
                const int stop = im ? __ffsll((long long)im) - 1 : 63;  // lanes 0..stop are needed
                const unsigned long long need = stop == 63 ? ~0ull : ((1ull << (stop + 1)) - 1);
                if (CBF_SCAN_TEST_TIMEOUT || (nr & need)) {
                    if (CBF_SCAN_TEST_TIMEOUT || ++spins > CBF_SCAN_SPIN_LIMIT) {
                        if (lane == 0) sctl[2] = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                int part = lane <= stop ? (int)(unsigned)(v & 0xFFFFFFFFull) : 0;
                for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
                excl += part;
                if (im) break;
                top -= 64;
            }
            if (lane == 0) st_state(&tstate[tile], ep | kFlagInc | (unsigned)(excl + agg));
        }
        if (lane == 0) {
            s_excl = excl;
            if (tile == ntiles - 1) start[ncell] = excl + agg;
        }
    }
    __syncthreads();
    int wpre = 0;
    for (int w = 0; w < wid; ++w) wpre += wtot[w];
    int run = s_excl + wpre + inc - tot;
    if (base + kPer <= ncell) {  // full tile: the lane's starts as 16-B stores, like the loads
        int o[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            o[k] = run;
            run += c[k];
        }
#pragma unroll
        for (int v = 0; v < kPer / 4; ++v)
            *reinterpret_cast<int4*>(start + base + 4 * v) = make_int4(o[4 * v], o[4 * v + 1], o[4 * v + 2], o[4 * v + 3]);
        return;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (base + k < ncell) start[base + k] = run;
        run += c[k];
    }
}

// Scatter into the cell-sorted copies.  Skipped entirely when the build is flagged unusable
// (sctl[2]: the starts cannot be trusted), and every slot is bounds-checked.
__global__ void __launch_bounds__(kBlock) k_scatter(int n, const int2* __restrict__ cs,
                                                    const int32_t* __restrict__ start,
                                                    const double2* __restrict__ pos, const double2* __restrict__ vel,
                                                    double2* __restrict__ spos, double2* __restrict__ svel,
                                                    int32_t* __restrict__ sidx, const int32_t* __restrict__ sctl) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || sctl[2] != 0) return;
    const int2 c = cs[i];
    if (c.x < 0) return;
    const int d = start[c.x] + c.y;
    if (d < 0 || d >= n) return;
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
                       W.sidx, W.sctl);
    return (int)hipGetLastError();
}

int build_cells(const CellGrid& G, const CellWs& W, int n, const double2* pos, const double2* vel, const int32_t*,
                hipStream_t s) {
    hipLaunchKernelGGL(k_bin, dim3(nblk(n)), dim3(kBlock), 0, s, G, n, pos, W.count, W.cs, W.sctl);
    return scan_and_scatter(G, W, n, pos, vel, s);
}

}  // namespace cbf
