// cells.hpp -- uniform cell list (counting sort by cell) shared by the swarm kernels.
//
// Build = bin (cell id + per-cell atomic slot) -> per-tile reduce -> tile scan -> scatter into
// cell-sorted SoA copies.  Slot order inside a cell depends on atomic arrival, which is harmless:
// the filter's per-quadrant minimum is order-independent, so results stay deterministic.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cbf_amd.h"

namespace cbf {

#ifndef CBF_SCAN_PER
#define CBF_SCAN_PER 8  // cells per scan lane (a multiple of 4)
#endif
constexpr int kScanTile = 256 * CBF_SCAN_PER;  // 256 threads x CBF_SCAN_PER cells
#ifndef CBF_HARD_BLOCKS
#define CBF_HARD_BLOCKS 128
#endif
// grid (64-lane blocks) of the hard-QP kernel of the lattice step: 8 k lanes cover the ~3 k queued
// QPs of cfg4 one per lane; each block ends with an atomic on the done counter, so fewer blocks
// end sooner (advance 50.2 us at 128 blocks, 51.0 at 256, 59.8 at 1024; tools/ablate.py set hard)
constexpr int kHardBlocks = CBF_HARD_BLOCKS;
constexpr int kHardHeader = 16;  // int32 words ahead of the hard-QP records (count + padding)

// A QP the filter kernel could not solve at the origin, queued with its assembled state.
struct HardRec {
    double r0, r1, r2, r3, u0x, u0y, bq0, bq1, bq2, bq3;
    int present, count, k, row;
};

struct CellGrid {
    double x0, y0, inv_h;
    int nx, ny;
};

inline CellGrid make_grid(const cbf_grid* g) {
    CellGrid G;
    G.x0 = g->x0;
    G.y0 = g->y0;
    G.inv_h = g->inv_h;
    G.nx = g->nx;
    G.ny = g->ny;
    return G;
}

inline size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

// Workspace carve-up (all segments 256-byte aligned).
struct CellWs {
    int32_t* count;   // [ncell]
    int32_t* start;   // [ncell + 1]
    unsigned long long* tstate;  // [ntiles] scan tile status {epoch:30 | flag:2 | value:32}
    int32_t* sctl;    // [64] scan control: [0] finished-tile counter, [1] epoch, [2] error flag
    int2* cs;        // [n] (cell, slot), cell < 0: not binned; 16 B/entry reserved (lattice: int4)
    double2* spos;    // [n] cell-sorted positions
    double2* svel;    // [n] cell-sorted velocities / nominal controls
    int32_t* sidx;    // [n] entity index of each sorted slot
    double2* wvel;    // [n] scratch velocities (lattice step: nominal of window agents)
    float2* spos32;   // [n] fp32 copy of spos (lattice step: the filter's distance screen)
    int32_t* hardq;   // lattice step: [0] = count, records (HardRec) from word kHardHeader
    long ncell;
    int ntiles;

    static int tiles(long ncell) { return (int)((ncell + kScanTile - 1) / kScanTile); }
    static size_t bytes(long n, long ncell) {
        return align256(4 * ncell) + align256(4 * (ncell + 1)) + align256(8 * (size_t)tiles(ncell)) + 256 +
               align256(16 * n) + 2 * align256(16 * n) + align256(4 * n) + align256(16 * n) + align256(8 * n) +
               align256(4 * kHardHeader + sizeof(HardRec) * (size_t)n);
    }
    CellWs(void* base, long n, long nc) : ncell(nc), ntiles(tiles(nc)) {
        char* p = (char*)base;
        count = (int32_t*)p;
        p += align256(4 * nc);
        start = (int32_t*)p;
        p += align256(4 * (nc + 1));
        tstate = (unsigned long long*)p;
        p += align256(8 * (size_t)ntiles);
        sctl = (int32_t*)p;
        p += 256;
        cs = (int2*)p;
        p += align256(16 * n);
        spos = (double2*)p;
        p += align256(16 * n);
        svel = (double2*)p;
        p += align256(16 * n);
        sidx = (int32_t*)p;
        p += align256(4 * n);
        wvel = (double2*)p;
        p += align256(16 * n);
        spos32 = (float2*)p;
        p += align256(8 * n);
        hardq = (int32_t*)p;
    }
};

// Full build from positions: memset counts, bin, scan, scatter (vel copied alongside).
// When `skip_bin` is set the caller already binned (count / cs filled by its own kernel).
int build_cells(const CellGrid& G, const CellWs& W, int n, const double2* pos, const double2* vel,
                const int32_t* unused, hipStream_t s);
int scan_and_scatter(const CellGrid& G, const CellWs& W, int n, const double2* pos, const double2* vel,
                     hipStream_t s);
// Exclusive scan of W.count into W.start (and re-zeroes W.count).
void launch_scan(const CellWs& W, hipStream_t s);

// CBF_SCAN_EPOCH_BIN: the scan's tile-state epoch is advanced by thread 0 of the bin kernel that
// precedes every scan (stream order makes it visible), instead of by the last scan block to
// finish -- that needed a returning atomic on one counter from each of the ~270 scan blocks, a
// serialised chain at the end of the scan.
#ifndef CBF_SCAN_EPOCH_BIN
#define CBF_SCAN_EPOCH_BIN 1
#endif
__device__ __forceinline__ void scan_epoch_advance(int32_t* sctl) {
    sctl[1] = (sctl[1] + 1) & 0x3FFFFFFF;  // one thread, before the scan kernel starts
}

}  // namespace cbf
