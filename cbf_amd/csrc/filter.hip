// filter.hip -- batched CBF safety filter kernels (gfx950):
//   get_safe_control over explicit neighbour lists   (cbf.py:18-92)
//   (A, b) row assembly                              (cbf.py:38-80)
//   all-pairs cull + filter, LDS-tiled               (cross_and_rescue.py:135-160)
//   cell-list cull + filter                          (same loop, O(N k))
#include "cbf_device.hpp"
#include "cells.hpp"

using namespace cbf;

namespace {

__global__ void __launch_bounds__(kBlock) k_safe_control_batch(KP P, int n, const double* __restrict__ rs,
                                                               const double* __restrict__ u0,
                                                               const int32_t* __restrict__ off,
                                                               const double* __restrict__ obs, double* __restrict__ u,
                                                               int32_t* __restrict__ status, double* __restrict__ xo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2 ra = reinterpret_cast<const double2*>(rs)[2 * i];
    const double2 rb = reinterpret_cast<const double2*>(rs)[2 * i + 1];
    const double2 uu = reinterpret_cast<const double2*>(u0)[i];
    Ego E;
    ego_init(P, E, ra.x, ra.y, rb.x, rb.y, uu.x, uu.y);
    const int t0 = off[i], t1 = off[i + 1];
    for (int t = t0; t < t1; ++t) {
        const double2 oa = reinterpret_cast<const double2*>(obs)[2 * t];
        const double2 ob = reinterpret_cast<const double2*>(obs)[2 * t + 1];
        ego_add(P, E, oa.x, oa.y, ob.x, ob.y);
    }
    const Sol S = solve_ego(P, E);
    double ux, uy;
    clip_u(P, S, E, ux, uy);
    reinterpret_cast<double2*>(u)[i] = make_double2(ux, uy);
    status[i] = pack_status(S);
    if (xo) reinterpret_cast<double2*>(xo)[i] = make_double2(S.x0, S.x1);
}

__global__ void __launch_bounds__(kBlock) k_assemble_rows(KP P, int n, const double* __restrict__ rs,
                                                          const double* __restrict__ u0,
                                                          const int32_t* __restrict__ off,
                                                          const double* __restrict__ obs, double* __restrict__ A,
                                                          double* __restrict__ b) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ego E;
    ego_init(P, E, rs[4 * i], rs[4 * i + 1], rs[4 * i + 2], rs[4 * i + 3], u0[2 * i], u0[2 * i + 1]);
    const int t0 = off[i], t1 = off[i + 1];
    const long base = (long)t0 + 8l * i;
    for (int t = t0; t < t1; ++t) {
        int q;
        const double bb = row_b(P, E, obs[4 * t], obs[4 * t + 1], obs[4 * t + 2], obs[4 * t + 3], q);
        double a0 = 0, a1 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (q == k) {
                a0 = P.n0[k];
                a1 = P.n1[k];
            }
        const long r = base + (t - t0);
        A[2 * r] = a0;
        A[2 * r + 1] = a1;
        b[r] = bb;
    }
    const Box B = box_rhs(P, E);
    const double g0[8] = {1.0, 0.0, -1.0, 0.0, 1.0, -1.0, 0.0, 0.0};
    const double g1[8] = {0.0, 1.0, 0.0, -1.0, 0.0, 0.0, 1.0, -1.0};
    const long rb = base + (t1 - t0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        A[2 * (rb + k)] = g0[k];
        A[2 * (rb + k) + 1] = g1[k];
        b[rb + k] = B.S[k];
    }
}

// Diagnostics shared by the swarm filters: neighbour rows re-evaluated at x from the recorded list.
__device__ void write_diag(const KP& P, const Ego& E, const Sol& S, int k, const double2* __restrict__ pos,
                           const double2* __restrict__ vel, const cbf_diag& D) {
    if (D.x) reinterpret_cast<double2*>(D.x)[k] = make_double2(S.x0, S.x1);
    if (D.viol) D.viol[k] = (E.count > 0) ? S.viol : 0.0;
    if (D.box_active) D.box_active[k] = (E.count > 0) ? box_active_bits(P, E, S) : 0;
    if (D.nbr_active && D.nbr_idx) {
        for (int t = 0; t < D.kmax; ++t) {
            const int j = D.nbr_idx[(long)k * D.kmax + t];
            uint8_t a = 0;
            if (j >= 0 && E.count > 0) {
                const double2 pj = pos[j], vj = vel[j];
                a = row_active(P, E, S, pj.x, pj.y, vj.x, vj.y);
            }
            D.nbr_active[(long)k * D.kmax + t] = a;
        }
    }
}

__device__ __forceinline__ void finish_ego(const KP& P, const Ego& E, int k, double* __restrict__ u,
                                           int32_t* __restrict__ status, int32_t* __restrict__ cnt, Sol& S) {
    double ux, uy;
    if (E.count == 0) {  // cross_and_rescue.py:153: filter not called, u0 kept unclipped
        ux = E.u0x;
        uy = E.u0y;
        S.status = CBF_STATUS_IDLE;
        S.iters = 0;
        S.x0 = S.x1 = 0.0;
        S.viol = 0.0;
    } else {
        S = solve_ego(P, E);
        clip_u(P, S, E, ux, uy);
    }
    reinterpret_cast<double2*>(u)[k] = make_double2(ux, uy);
    status[k] = (E.count == 0) ? CBF_STATUS_IDLE : pack_status(S);
    if (cnt) cnt[k] = E.count;
}

__device__ __forceinline__ double absmax2(double2 p) { return pmax(fabs(p.x), fabs(p.y)); }

// exact cull test (fp64) + row assembly of staged candidate t (entity base + t)
__device__ __forceinline__ void ap_exact(const KP& P, Ego& E, const double2* sp, const double2* sv, int base, int t,
                                         int n_obs, const cbf_diag& D, int k, int& recorded) {
    const double2 pj = sp[t];
    double s;
    if (cull_keep(P, E.r0, E.r1, pj.x, pj.y, base + t < n_obs, s)) {
        const double2 vj = sv[t];
        ego_add(P, E, pj.x, pj.y, vj.x, vj.y);
        if (D.nbr_idx && recorded < D.kmax) D.nbr_idx[(long)k * D.kmax + recorded++] = base + t;
    }
}

#ifndef CBF_AP_TILE
#define CBF_AP_TILE 256   // candidates staged per tile (a multiple of kBlock)
#endif
// CBF_AP_WPE: test build only (tests/_lib/libcbf_apwpe8.so, tests/test_gpu_parity.py): an
// occupancy request on the all-pairs kernels that forces register spilling, kept to re-check that
// the spilled code stays bit-identical (negative results).
#ifdef CBF_AP_WPE
#define CBF_AP_OCC __attribute__((amdgpu_waves_per_eu(CBF_AP_WPE, CBF_AP_WPE)))
#else
#define CBF_AP_OCC
#endif
#ifndef CBF_AP_SCREEN
#define CBF_AP_SCREEN 8   // candidates per screen step
#endif

// The all-pairs candidate loop of one ego over entities [c0, c1): tiles of CBF_AP_TILE entities
// staged in LDS (fp64 state plus fp32 copies of the positions, SoA, so one 16-B LDS read brings 4
// consecutive candidates) and read by broadcast (every lane reads the same
// candidate), ascending index order (= reference order).  CBF_AP_SCREEN candidates per screen
// step; the exact test and row assembly run only for candidates the screen lets through.  Every
// lane of the block must call it (it synchronises the block).
struct ApLds {
    double2 sp[CBF_AP_TILE];
    double2 sv[CBF_AP_TILE];
    float xs32[CBF_AP_TILE];
    float ys32[CBF_AP_TILE];
    double smax[kBlock / 64];
};

template <class Hit>
__device__ __forceinline__ void allpairs_scan(const KP& P, double r0, double r1, bool active, int c0, int c1,
                                              const double2* __restrict__ pos, const double2* __restrict__ vel,
                                              ApLds& L, Hit& hit) {
    constexpr int kScreen = CBF_AP_SCREEN;
    constexpr int kTile = CBF_AP_TILE;
    constexpr int kPer = kTile / kBlock;
    const float ex = (float)r0, ey = (float)r1;
    double m_ego = absmax2(make_double2(r0, r1));
    if (m_ego != m_ego) m_ego = INFINITY;
    for (int base = c0; base < c1; base += kTile) {
        double mj = 0.0;
#pragma unroll
        for (int c = 0; c < kPer; ++c) {
            const int tl = c * kBlock + threadIdx.x;
            const int j = base + tl;
            if (j < c1) {
                const double2 pj = pos[j];
                L.sp[tl] = pj;
                L.sv[tl] = vel[j];
                const float x = (float)pj.x, y = (float)pj.y;
                L.xs32[tl] = x;
                L.ys32[tl] = y;
                double a = absmax2(pj);
                if (a != a) a = INFINITY;  // NaN coordinate: screen off for this tile
                mj = pmax(mj, a);
            }
        }
        for (int o = 32; o > 0; o >>= 1) mj = pmax(mj, __shfl_xor(mj, o, 64));
        if ((threadIdx.x & 63) == 0) L.smax[threadIdx.x >> 6] = mj;
        __syncthreads();
        const int m = min(kTile, c1 - base);
        if (active) {
            double mt = L.smax[0];
#pragma unroll
            for (int w = 1; w < kBlock / 64; ++w) mt = pmax(mt, L.smax[w]);
            const double M = pmax(mt, m_ego);
            int t = 0;
            // fp32 difference-form screen; it only rejects (screen_threshold), and it is off for
            // tiles with huge or non-finite coordinates (every candidate then takes the exact test)
            const float t32 = screen_threshold(P.cull_t, M);
            if (t32 > 0.0f) {
                for (; t + kScreen <= m; t += kScreen) {
                    float sq[kScreen];
#pragma unroll
                    for (int q = 0; q < kScreen; q += 4) {
                        const float4 X = *reinterpret_cast<const float4*>(&L.xs32[t + q]);
                        const float4 Y = *reinterpret_cast<const float4*>(&L.ys32[t + q]);
                        const float xs[4] = {X.x, X.y, X.z, X.w}, ys[4] = {Y.x, Y.y, Y.z, Y.w};
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const float d0 = xs[k] - ex, d1 = ys[k] - ey;
                            sq[q + k] = __builtin_fmaf(d0, d0, d1 * d1);
                        }
                    }
                    float mn = sq[0];
#pragma unroll
                    for (int q = 1; q < kScreen; ++q) mn = fminf(mn, sq[q]);
                    if (mn < t32) {
#pragma unroll
                        for (int q = 0; q < kScreen; ++q)
                            if (sq[q] < t32) hit(base, t + q);
                    }
                }
            }
            for (; t < m; ++t) hit(base, t);
        }
        __syncthreads();
    }
}

// hit visitors of allpairs_scan (called for candidates the screen lets through)
struct HitAssemble {  // exact test + row assembly into the ego's QP (+ neighbour list)
    const KP& P;
    Ego& E;
    const ApLds& L;
    int n_obs;
    const cbf_diag& D;
    int k;
    int recorded;
    __device__ __forceinline__ void operator()(int base, int t) {
        ap_exact(P, E, L.sp, L.sv, base, t, n_obs, D, k, recorded);
    }
};
struct HitRecord {  // exact test only: neighbour indices (first kmax, ascending) and count
    const KP& P;
    const ApLds& L;
    double r0, r1;
    int n_obs;
    int32_t* idx;
    int kmax;
    int count;
    __device__ __forceinline__ void operator()(int base, int t) {
        const double2 pj = L.sp[t];
        double s;
        if (cull_keep(P, r0, r1, pj.x, pj.y, base + t < n_obs, s)) {
            if (count < kmax) idx[count] = base + t;
            ++count;
        }
    }
};

__global__ void __launch_bounds__(kBlock) CBF_AP_OCC k_filter_allpairs(KP P, int n, int n_obs, const double2* __restrict__ pos,
                                                            const double2* __restrict__ vel, int ego_begin,
                                                            int ego_end, double* __restrict__ u,
                                                            int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                            cbf_diag D) {
    __shared__ ApLds L;
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    const bool active = e < ego_end;
    Ego E;
    {
        const double2 pe = active ? pos[e] : make_double2(0, 0);
        const double2 ve = active ? vel[e] : make_double2(0, 0);
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    }
    const int k = e - ego_begin;
    HitAssemble hit{P, E, L, n_obs, D, k, 0};
    allpairs_scan(P, E.r0, E.r1, active, 0, n, pos, vel, L, hit);
    if (!active) return;
    if (D.nbr_idx)
        for (int t = hit.recorded; t < D.kmax; ++t) D.nbr_idx[(long)k * D.kmax + t] = -1;
    Sol S;
    finish_ego(P, E, k, u, status, cnt, S);
    write_diag(P, E, S, k, pos, vel, D);
}

// All-pairs cull only (cross_and_rescue.py:141-150): per ego the first kmax neighbour indices in
// reference order (obstacles, then agents, ascending) and the full count.
__global__ void __launch_bounds__(kBlock) CBF_AP_OCC k_cull_allpairs(KP P, int n, int n_obs, const double2* __restrict__ pos,
                                                          int ego_begin, int ego_end, int kmax,
                                                          int32_t* __restrict__ nbr_idx,
                                                          int32_t* __restrict__ nbr_count) {
    __shared__ ApLds L;
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    const bool active = e < ego_end;
    const double2 pe = active ? pos[e] : make_double2(0, 0);
    const long k = e - ego_begin;
    HitRecord hit{P, L, pe.x, pe.y, n_obs, nbr_idx + k * kmax, kmax, 0};
    allpairs_scan(P, pe.x, pe.y, active, 0, n, pos, pos, L, hit);
    if (!active) return;
    for (int t = hit.count; t < kmax; ++t) nbr_idx[k * kmax + t] = -1;
    nbr_count[k] = hit.count;
}

// Split all-pairs: workgroup (x, y) runs egos [x*kBlock, ...) against candidate chunk y and
// leaves the chunk's partial QP state; k_allpairs_finish merges the chunks in order.  The
// per-quadrant minimum ignores NaN rows whatever the order, so merging is exact.
struct ApPart {
    double bq0, bq1, bq2, bq3;
    int present, count;
};

inline int ap_chunks(long n, long n_ego) {
    const long ego_waves = (n_ego + 63) / 64;
    long s = (8192 + ego_waves - 1) / (ego_waves > 0 ? ego_waves : 1);  // ~8 waves per SIMD
    const long smax = (n + 2047) / 2048;                                 // >= 2048 candidates per chunk
    if (s > smax) s = smax;
    return (int)(s < 1 ? 1 : s);
}
inline long ap_chunk_len(long n, int s) {
    const long c = (n + s - 1) / s;
    return (c + CBF_AP_TILE - 1) / CBF_AP_TILE * CBF_AP_TILE;
}

__global__ void __launch_bounds__(kBlock) CBF_AP_OCC k_allpairs_partial(KP P, int n, int n_obs, const double2* __restrict__ pos,
                                                             const double2* __restrict__ vel, int ego_begin,
                                                             int ego_end, int chunk, ApPart* __restrict__ part) {
    __shared__ ApLds L;
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    const bool active = e < ego_end;
    Ego E;
    {
        const double2 pe = active ? pos[e] : make_double2(0, 0);
        const double2 ve = active ? vel[e] : make_double2(0, 0);
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    }
    const int c0 = blockIdx.y * chunk;
    const int c1 = min(n, c0 + chunk);
    const int k = e - ego_begin;
    const cbf_diag D0 = {};
    HitAssemble hit{P, E, L, n_obs, D0, k, 0};
    allpairs_scan(P, E.r0, E.r1, active, c0, c1, pos, vel, L, hit);
    if (!active) return;
    ApPart o;
    o.bq0 = E.bq0;
    o.bq1 = E.bq1;
    o.bq2 = E.bq2;
    o.bq3 = E.bq3;
    o.present = (int)E.present;
    o.count = E.count;
    part[(long)blockIdx.y * (ego_end - ego_begin) + k] = o;
}

__global__ void __launch_bounds__(kBlock) CBF_AP_OCC k_allpairs_finish(KP P, int nchunk, const double2* __restrict__ pos,
                                                            const double2* __restrict__ vel, int ego_begin,
                                                            int ego_end, const ApPart* __restrict__ part,
                                                            double* __restrict__ u, int32_t* __restrict__ status,
                                                            int32_t* __restrict__ cnt) {
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    if (e >= ego_end) return;
    const int k = e - ego_begin;
    const long ne = ego_end - ego_begin;
    const double2 pe = pos[e], ve = vel[e];
    Ego E;
    ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    for (int c = 0; c < nchunk; ++c) {
        const ApPart o = part[c * ne + k];
        E.bq0 = pmin(E.bq0, o.bq0);
        E.bq1 = pmin(E.bq1, o.bq1);
        E.bq2 = pmin(E.bq2, o.bq2);
        E.bq3 = pmin(E.bq3, o.bq3);
        E.present |= (unsigned)o.present;
        E.count += o.count;
    }
    Sol S;
    finish_ego(P, E, k, u, status, cnt, S);
}

// Cell-list filter over sorted slots: lane = sorted slot (spatially coherent waves).
__global__ void __launch_bounds__(kBlock) k_filter_cells(KP P, CellGrid G, int n, int n_obs,
                                                         const double2* __restrict__ spos,
                                                         const double2* __restrict__ svel,
                                                         const int32_t* __restrict__ sidx,
                                                         const int32_t* __restrict__ start, int ego_begin,
                                                         int ego_end, double* __restrict__ u,
                                                         int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                         const double2* __restrict__ pos,
                                                         const double2* __restrict__ vel, cbf_diag D,
                                                         const int32_t* __restrict__ sctl) {
    const int slot = blockIdx.x * kBlock + threadIdx.x;
    if (slot >= n) return;
    if (sctl[2] != 0) {  // the cell list of this call is unusable (cells.hpp build_begin, cells.hip scan):
        const int e = slot;  // touch none of it; every ego reports the error, unfiltered
        if (e < ego_begin || e >= ego_end) return;
        const int k = e - ego_begin;
        reinterpret_cast<double2*>(u)[k] = vel[e];
        status[k] = CBF_STATUS_WORKSPACE_ERROR;
        if (cnt) cnt[k] = 0;
        return;
    }
    const int e = sidx[slot];
    if (e < ego_begin || e >= ego_end) return;
    const double2 pe = spos[slot], ve = svel[slot];
    Ego E;
    ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    const int k = e - ego_begin;
    int recorded = 0;
    const int cx = cell_coord(pe.x, G.x0, G.inv_h, G.nx);
    const int cy = cell_coord(pe.y, G.y0, G.inv_h, G.ny);
    const int xa = cx > 0 ? cx - 1 : 0;
    const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = cy + dy;
        if (yy < 0 || yy >= G.ny) continue;
        const int t0 = start[yy * G.nx + xa], t1 = start[yy * G.nx + xb + 1];
        for (int t = t0; t < t1; ++t) {
            const double2 pj = spos[t];
            const double e0 = pj.x - E.r0, e1 = pj.y - E.r1;
            const double s = e0 * e0 + e1 * e1;
            if (!(s < P.cull_t)) continue;
            int j = -1;
            if (!(s > 0) || D.nbr_idx) j = sidx[t];
            if (!(s > 0) && j >= n_obs) continue;
            const double2 vj = svel[t];
            ego_add(P, E, pj.x, pj.y, vj.x, vj.y);
            if (D.nbr_idx && recorded < D.kmax) D.nbr_idx[(long)k * D.kmax + recorded++] = j;
        }
    }
    if (D.nbr_idx)
        for (int t = recorded; t < D.kmax; ++t) D.nbr_idx[(long)k * D.kmax + t] = -1;
    Sol S;
    finish_ego(P, E, k, u, status, cnt, S);
    write_diag(P, E, S, k, pos, vel, D);
}

inline int grid_for(long n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

extern "C" int cbf_get_safe_control_batch(const cbf_params* p, int32_t n_ego, const double* robot_state,
                                          const double* u0, const int32_t* nbr_off, const double* obs_states,
                                          double* u, int32_t* status, double* x_out, void* stream) {
    if (!p || n_ego < 0 || (n_ego > 0 && (!robot_state || !u0 || !nbr_off || !u || !status))) return CBF_EINVAL;
    if (n_ego == 0) return 0;
    hipLaunchKernelGGL(k_safe_control_batch, dim3(grid_for(n_ego)), dim3(kBlock), 0, (hipStream_t)stream,
                       make_kp(p), n_ego, robot_state, u0, nbr_off, obs_states, u, status, x_out);
    return (int)hipGetLastError();
}

extern "C" int cbf_assemble_rows(const cbf_params* p, int32_t n_ego, const double* robot_state, const double* u0,
                                 const int32_t* nbr_off, const double* obs_states, double* A, double* b,
                                 void* stream) {
    if (!p || n_ego < 0 || (n_ego > 0 && (!robot_state || !u0 || !nbr_off || !A || !b))) return CBF_EINVAL;
    if (n_ego == 0) return 0;
    hipLaunchKernelGGL(k_assemble_rows, dim3(grid_for(n_ego)), dim3(kBlock), 0, (hipStream_t)stream, make_kp(p),
                       n_ego, robot_state, u0, nbr_off, obs_states, A, b);
    return (int)hipGetLastError();
}

static int check_swarm_args(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos, const double* vel,
                            int32_t ego_begin, int32_t ego_end, double* u, int32_t* status, const cbf_diag* diag) {
    if (!p || n < 0 || n_obs < 0 || n_obs > n || ego_begin < n_obs || ego_end > n || ego_begin > ego_end)
        return CBF_EINVAL;
    if (n > 0 && (!pos || !vel)) return CBF_EINVAL;
    if (ego_end > ego_begin && (!u || !status)) return CBF_EINVAL;
    if (diag && diag->kmax < 0) return CBF_EINVAL;
    if (diag && diag->nbr_active && !diag->nbr_idx) return CBF_EINVAL;
    return 0;
}

static cbf_diag diag_or_empty(const cbf_diag* d) {
    cbf_diag D;
    if (d) {
        D = *d;
        if (D.kmax == 0) D.nbr_idx = nullptr, D.nbr_active = nullptr;
    } else {
        D.kmax = 0;
        D.nbr_idx = nullptr;
        D.nbr_active = nullptr;
        D.box_active = nullptr;
        D.x = nullptr;
        D.viol = nullptr;
    }
    return D;
}

extern "C" int cbf_filter_allpairs(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos,
                                   const double* vel, int32_t ego_begin, int32_t ego_end, double* u, int32_t* status,
                                   int32_t* nbr_count, const cbf_diag* diag, void* stream) {
    const int rc = check_swarm_args(p, n, n_obs, pos, vel, ego_begin, ego_end, u, status, diag);
    if (rc) return rc;
    const int ne = ego_end - ego_begin;
    if (ne == 0) return 0;
    hipLaunchKernelGGL(k_filter_allpairs, dim3(grid_for(ne)), dim3(kBlock), 0, (hipStream_t)stream, make_kp(p), n,
                       n_obs, reinterpret_cast<const double2*>(pos), reinterpret_cast<const double2*>(vel),
                       ego_begin, ego_end, u, status, nbr_count, diag_or_empty(diag));
    return (int)hipGetLastError();
}

extern "C" int cbf_cull_allpairs(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos, int32_t ego_begin,
                                 int32_t ego_end, int32_t kmax, int32_t* nbr_idx, int32_t* nbr_count, void* stream) {
    if (!p || n < 0 || n_obs < 0 || n_obs > n || ego_begin < n_obs || ego_end > n || ego_begin > ego_end || kmax < 0)
        return CBF_EINVAL;
    const int ne = ego_end - ego_begin;
    if (ne == 0) return 0;
    if (!pos || !nbr_count || (kmax > 0 && !nbr_idx)) return CBF_EINVAL;
    hipLaunchKernelGGL(k_cull_allpairs, dim3(grid_for(ne)), dim3(kBlock), 0, (hipStream_t)stream, make_kp(p), n, n_obs,
                       reinterpret_cast<const double2*>(pos), ego_begin, ego_end, kmax, nbr_idx, nbr_count);
    return (int)hipGetLastError();
}

extern "C" size_t cbf_allpairs_workspace_size(int32_t n, int32_t n_ego) {
    if (n < 0 || n_ego < 0) return 0;
    return align256(sizeof(ApPart) * (size_t)ap_chunks(n, n_ego) * (size_t)(n_ego > 0 ? n_ego : 1));
}

extern "C" int cbf_filter_allpairs_split(const cbf_params* p, int32_t n, int32_t n_obs, const double* pos,
                                         const double* vel, int32_t ego_begin, int32_t ego_end, double* u,
                                         int32_t* status, int32_t* nbr_count, void* workspace, size_t workspace_bytes,
                                         void* stream) {
    const int rc = check_swarm_args(p, n, n_obs, pos, vel, ego_begin, ego_end, u, status, nullptr);
    if (rc) return rc;
    const int ne = ego_end - ego_begin;
    if (ne == 0) return 0;
    if (!workspace || workspace_bytes < cbf_allpairs_workspace_size(n, ne)) return CBF_EINVAL;
    const int s = ap_chunks(n, ne);
    const long chunk = ap_chunk_len(n, s);
    const KP kp = make_kp(p);
    ApPart* part = reinterpret_cast<ApPart*>(workspace);
    hipStream_t st = (hipStream_t)stream;
    const double2* p2 = reinterpret_cast<const double2*>(pos);
    const double2* v2 = reinterpret_cast<const double2*>(vel);
    hipLaunchKernelGGL(k_allpairs_partial, dim3(grid_for(ne), s), dim3(kBlock), 0, st, kp, n, n_obs, p2, v2,
                       ego_begin, ego_end, (int)chunk, part);
    hipLaunchKernelGGL(k_allpairs_finish, dim3(grid_for(ne)), dim3(kBlock), 0, st, kp, s, p2, v2, ego_begin, ego_end,
                       part, u, status, nbr_count);
    return (int)hipGetLastError();
}

extern "C" size_t cbf_cells_workspace_size(int32_t n, const cbf_grid* grid) {
    if (!grid || n < 0 || grid->nx <= 0 || grid->ny <= 0) return 0;
    return CellWs::bytes(n, (long)grid->nx * grid->ny);
}

extern "C" int cbf_filter_cells(const cbf_params* p, const cbf_grid* grid, int32_t n, int32_t n_obs,
                                const double* pos, const double* vel, int32_t ego_begin, int32_t ego_end, double* u,
                                int32_t* status, int32_t* nbr_count, const cbf_diag* diag, void* workspace,
                                size_t workspace_bytes, void* stream) {
    int rc = check_swarm_args(p, n, n_obs, pos, vel, ego_begin, ego_end, u, status, diag);
    if (rc) return rc;
    if (!grid || grid->nx <= 0 || grid->ny <= 0 || !(grid->inv_h > 0)) return CBF_EINVAL;
    if (!(1.0 / grid->inv_h >= sqrt(p->cull_t))) return CBF_EINVAL;  // cell edge must cover the cull radius
    if ((long)grid->nx * grid->ny > (1l << 30)) return CBF_EINVAL;
    if (n == 0 || ego_end == ego_begin) return 0;
    if (!workspace || workspace_bytes < cbf_cells_workspace_size(n, grid)) return CBF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const CellGrid G = make_grid(grid);
    CellWs W(workspace, n, (long)G.nx * G.ny);
    rc = build_cells(G, W, n, reinterpret_cast<const double2*>(pos), reinterpret_cast<const double2*>(vel),
                     nullptr, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_filter_cells, dim3(grid_for(n)), dim3(kBlock), 0, s, make_kp(p), G, n, n_obs, W.spos, W.svel,
                       W.sidx, W.start, ego_begin, ego_end, u, status, nbr_count,
                       reinterpret_cast<const double2*>(pos), reinterpret_cast<const double2*>(vel),
                       diag_or_empty(diag), W.sctl);
    return (int)hipGetLastError();
}
