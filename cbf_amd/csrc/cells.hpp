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
#define CBF_SCAN_PER 8  // cells per scan lane
#endif
static_assert(CBF_SCAN_PER >= 4 && CBF_SCAN_PER % 4 == 0, "the scan moves its cells as 16-B int4 vectors");
constexpr int kScanTile = 256 * CBF_SCAN_PER;  // 256 threads x CBF_SCAN_PER cells
// Hard-QP queues of the lattice step: kSubQ sub-queues; filter block b appends the QPs it cannot
// finish at the origin to sub-queue b % kSubQ (one wave-aggregated atomic per wave on that
// sub-queue's counter), so the entries of a sub-queue are contiguous and the queue kernel runs
// them in full waves.  One chip-wide counter serialised ~16 k wave atomics a step at the memory
// side (the filter ran 200 us instead of 43 at cfg4f); 64 counters on separate 128-B lines take
// ~256 each, in parallel.  Header: [2..7] the cell-order state of the last build; [32 (1 + q)]
// sub-queue q's length; [32 (1 + kSubQ + q)] its done counter (queue kernel).
constexpr int kSubQ = 64;
constexpr int kHardHeader = 32 * (1 + 2 * kSubQ);
// A QP the filter kernel could not solve at the origin, queued with its assembled state.
struct HardRec {
    double r0, r1, r2, r3, u0x, u0y, bq0, bq1, bq2, bq3;
    int present, count, k, row, slot;  // row: window index of the agent; slot: its cell-sorted slot
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

// Workspace carve-up (all segments 256-byte aligned).  The control words come first, at a fixed
// offset, so that the shape signature they hold can be checked whatever shape a call assumes.
struct CellWs {
    int32_t* sctl;    // [64] control: [1] scan epoch, [2] error flag of this build (scan look-back
                      // gave up, or workspace shape mismatch), [4] n, [5] ncell: the shape the
                      // workspace is bound to (0 = fresh); [8] lattice nominal-control mode, bytes
                      // 40..55 its amplitude (double) and seed (uint64) (cbf_lattice_set_nominal)
    int32_t* count;   // [ncell]
    int32_t* start;   // [ncell + 1]
    unsigned long long* tstate;  // [ntiles] scan tile status {epoch:30 | flag:2 | value:32}
    int2* cs;         // [n] (cell, slot), cell < 0: not binned; 16 B/entry reserved (lattice: int3)
    double2* spos;    // [n] cell-sorted positions
    double2* svel;    // [n] cell-sorted velocities / nominal controls
    int32_t* sidx;    // [n] entity index of each sorted slot
    double2* wvel;    // [n] scratch velocities
    int32_t* hardq;   // lattice step: header (kHardHeader words)
    HardRec* qrec;    // [kSubQ * qcap] sub-queue q at qrec + q * qcap (HOCBF: int slots)
    long ncell;
    int ntiles;
    long qcap;

    static int tiles(long ncell) { return (int)((ncell + kScanTile - 1) / kScanTile); }
    // capacity of a sub-queue: the egos of the filter blocks that append to it
    static long subq_cap(long n) { return ((n + kBlock - 1) / kBlock + kSubQ - 1) / kSubQ * kBlock; }
    static size_t bytes(long n, long ncell) {
        return 256 + align256(4 * ncell) + align256(4 * (ncell + 1)) + align256(8 * (size_t)tiles(ncell)) +
               align256(16 * n) + 2 * align256(16 * n) + align256(4 * n) + align256(16 * n) +
               align256(4 * kHardHeader) + align256(sizeof(HardRec) * (size_t)(kSubQ * subq_cap(n)));
    }
    CellWs(void* base, long n, long nc) : ncell(nc), ntiles(tiles(nc)), qcap(subq_cap(n)) {
        char* p = (char*)base;
        sctl = (int32_t*)p;
        p += 256;
        count = (int32_t*)p;
        p += align256(4 * nc);
        start = (int32_t*)p;
        p += align256(4 * (nc + 1));
        tstate = (unsigned long long*)p;
        p += align256(8 * (size_t)ntiles);
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
        hardq = (int32_t*)p;
        p += align256(4 * kHardHeader);
        qrec = (HardRec*)p;
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

// Start of a build, by thread 0 of the bin kernel that precedes every scan (stream order makes it
// visible): advance the scan's tile-state epoch (rather than by the last scan block to finish,
// which needed a returning atomic from each of the ~270 scan blocks: a serialised chain), clear
// the error flag, and check the workspace's shape binding.  A workspace holds counts, starts and
// tile words whose offsets depend on (n, ncell); reused for another shape without re-zeroing, those
// would corrupt the cell list, so a mismatch sets the error flag (every ego of the step reports
// CBF_STATUS_WORKSPACE_ERROR) and stays bound to the old shape, so later calls fail the same way
// until the caller zero-fills the workspace.
// The lattice nominal-control spec in a workspace's control words (cbf_lattice_set_nominal):
// mode 0 (the zero-filled default) = lattice-Laplacian consensus with the call's gain.
struct NominalSpec {
    int mode;
    double amp;
    unsigned long long seed;
};
__device__ __forceinline__ NominalSpec nominal_spec(const int32_t* sctl) {
    NominalSpec N;
    N.mode = sctl[8];
    N.amp = reinterpret_cast<const double*>(sctl)[5];
    N.seed = reinterpret_cast<const unsigned long long*>(sctl)[6];
    return N;
}

__device__ __forceinline__ void build_begin(int32_t* sctl, long n, long ncell) {
    sctl[1] = (sctl[1] + 1) & 0x3FFFFFFF;
    const bool fresh = sctl[4] == 0 && sctl[5] == 0;
    const bool same = sctl[4] == (int32_t)n && sctl[5] == (int32_t)ncell;
    sctl[2] = (fresh || same) ? 0 : 1;
    if (fresh) {
        sctl[4] = (int32_t)n;
        sctl[5] = (int32_t)ncell;
    }
}

}  // namespace cbf
