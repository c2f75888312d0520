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
// sub-queue q's length; [32 (1 + kSubQ + q)] its done counter (queue kernel); the same words + 16:
// the HOCBF step's second queue (hocbf.hip kHardQ2).
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

// Version of the workspace carve-up below and of its control words (cbf_workspace_layout): bump it
// with ANY change to CellWs, HardRec, the control-word assignments or the queue header, so that a
// saved workspace is never restored into a library that reads it differently.
constexpr int kWorkspaceLayout = 7;

// Workspace carve-up (all segments 256-byte aligned).  The control words come first, at a fixed
// offset, so that the shape signature they hold can be checked whatever shape a call assumes.
struct CellWs {
    int32_t* sctl;    // [64] control: [1] scan epoch, [2] error flag of this build (scan look-back
                      // gave up, or workspace shape mismatch), [4] n, [5] ncell: the shape the
                      // workspace is bound to (0 = fresh); [8] lattice nominal-control mode, bytes
                      // 40..55 its amplitude (double) and seed (uint64) (cbf_lattice_set_nominal);
                      // [16] the window cull's guard-token count, [17] the row-guard mode of
                      // its last build (window.hip kWinTokenWord / kWinModeWord); [20..21]
                      // (uint64) egos that took the window cull's unbounded walk and [22..23]
                      // (uint64) row-guard words read at their spin limit, both accumulated for
                      // the workspace's life and checkpointed with it (window.hip kWinWalkWord /
                      // kWinStallWord, cbf_lattice_window_counters)
    int32_t* count;   // [ncell]
    int32_t* start;   // [ncell + 1]
    unsigned long long* tstate;  // [ntiles] scan tile status {epoch:30 | flag:2 | value:32}
    int32_t* tdone;   // [ntiles] scan tile "starts written" words (tile_done_word(epoch))
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
               align256(4 * (size_t)tiles(ncell)) + align256(16 * n) + 2 * align256(16 * n) + align256(4 * n) + align256(16 * n) +
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
        tdone = (int32_t*)p;
        p += align256(4 * (size_t)ntiles);
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

// A 16-B write-through store (sc1: the line leaves the XCD's L2 for memory; MI355X_MICROARCH.md).
typedef int cbf_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_sc1_x4(int32_t* p, int4 v) {
    const cbf_v4i w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(w) : "memory");
}

// a tile's done word for scan epoch e: never 0, so a zero-filled workspace holds no done tile
__device__ __forceinline__ int32_t tile_done_word(unsigned e) { return (int32_t)((e & 0x3FFFFFFFu) | 0x40000000u); }

// `tdone` (may be null): tile -> its done word (tile_done_word(epoch)), published once the tile's
// starts are written, for a kernel that consumes the starts while the scan runs
// (k_lattice_scan_scatter).  The hand-off is the write-through (sc1) form of MI355X_MICROARCH.md
// (inter-workgroup visibility, the table's first row), NOT an agent-scope release/acquire pair:
// every start is stored with an sc1 store, every storing wave waits for its stores (vmcnt(0)),
// a block barrier, then ONE lane's sc1 done-word store; the consumer polls the word with sc1
// loads from one lane of the wave and that wave then reads the starts with sc1 loads only (no
// acquire fence: the loads bypass L1, and one invalidate per polling wave cost more than the
// launch this fusion saves).  tests/test_gpu_parity.py checks every start at full size against
// a host exclusive scan of the cell counts.  Every thread of the block must call it.
__device__ __forceinline__ void scan_tile(int32_t* __restrict__ count, long ncell, int ntiles,
                                          int32_t* __restrict__ start, unsigned long long* __restrict__ tstate,
                                          int32_t* __restrict__ sctl, int tile, int32_t* __restrict__ tdone) {
    __shared__ int s_excl;
    __shared__ int wtot[kBlock / 64];
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
                        if (lane == 0) __hip_atomic_store(&sctl[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
        for (int v = 0; v < kPer / 4; ++v) {
            const int4 w = make_int4(o[4 * v], o[4 * v + 1], o[4 * v + 2], o[4 * v + 3]);
            if (tdone)
                store_sc1_x4(start + base + 4 * v, w);
            else
                *reinterpret_cast<int4*>(start + base + 4 * v) = w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (base + k < ncell) {
                if (tdone)
                    __hip_atomic_store(&start[base + k], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    start[base + k] = run;
            }
            run += c[k];
        }
    }
    if (tdone) {
        // in-launch hand-off of the starts (the sc1 form above; relaxed agent-scope atomics lower
        // to sc1 loads / stores): write-through start stores, every storing wave waits for them, a
        // block barrier, then ONE lane's sc1 done-word store.  A timed-out look-back's error flag
        // is an sc1 store too.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(&tdone[tile], tile_done_word(epoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace cbf
