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

// Single-pass exclusive scan of the cell counts (decoupled look-back): scan_tile (cells.hpp), one
// tile per block.
__global__ void __launch_bounds__(kBlock) k_scan_onepass(int32_t* __restrict__ count, long ncell, int ntiles,
                                                         int32_t* __restrict__ start,
                                                         unsigned long long* __restrict__ tstate,
                                                         int32_t* __restrict__ sctl) {
    scan_tile(count, ncell, ntiles, start, tstate, sctl, (int)blockIdx.x, nullptr);
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

extern "C" int cbf_workspace_layout(void) { return cbf::kWorkspaceLayout; }

extern "C" int64_t cbf_lattice_workspace_view(int32_t W, int32_t win_rows, const cbf_grid* grid, int64_t* off) {
    if (!grid || !off || W <= 0 || win_rows <= 0 || grid->nx <= 0 || grid->ny <= 0) return CBF_EINVAL;
    const long n = (long)W * win_rows, ncell = (long)grid->nx * grid->ny;
    const uintptr_t base = 4096;  // the carve-up only adds offsets to its base
    cbf::CellWs Wk(reinterpret_cast<void*>(base), n, ncell);
    off[0] = (int64_t)(reinterpret_cast<uintptr_t>(Wk.start) - base);
    off[1] = (int64_t)(reinterpret_cast<uintptr_t>(Wk.spos) - base);
    off[2] = (int64_t)(reinterpret_cast<uintptr_t>(Wk.svel) - base);
    off[3] = (int64_t)(reinterpret_cast<uintptr_t>(Wk.sidx) - base);
    return ncell;
}
