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

// All-pairs: one lane per ego, candidate tiles of kBlock entities staged in LDS and read by
// broadcast (every lane reads the same candidate), ascending index order (= reference order).
__global__ void __launch_bounds__(kBlock) k_filter_allpairs(KP P, int n, int n_obs, const double2* __restrict__ pos,
                                                            const double2* __restrict__ vel, int ego_begin,
                                                            int ego_end, double* __restrict__ u,
                                                            int32_t* __restrict__ status, int32_t* __restrict__ cnt,
                                                            cbf_diag D) {
    __shared__ double2 sp[kBlock];
    __shared__ double2 sv[kBlock];
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    const bool active = e < ego_end;
    Ego E;
    {
        const double2 pe = active ? pos[e] : make_double2(0, 0);
        const double2 ve = active ? vel[e] : make_double2(0, 0);
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    }
    const int k = e - ego_begin;
    int recorded = 0;
    for (int base = 0; base < n; base += kBlock) {
        const int j = base + threadIdx.x;
        if (j < n) {
            sp[threadIdx.x] = pos[j];
            sv[threadIdx.x] = vel[j];
        }
        __syncthreads();
        const int m = min(kBlock, n - base);
        if (active) {
            for (int t = 0; t < m; ++t) {
                const double2 pj = sp[t];
                double s;
                if (cull_keep(P, E.r0, E.r1, pj.x, pj.y, base + t < n_obs, s)) {
                    const double2 vj = sv[t];
                    ego_add(P, E, pj.x, pj.y, vj.x, vj.y);
                    if (D.nbr_idx && recorded < D.kmax) D.nbr_idx[(long)k * D.kmax + recorded++] = base + t;
                }
            }
        }
        __syncthreads();
    }
    if (!active) return;
    if (D.nbr_idx)
        for (int t = recorded; t < D.kmax; ++t) D.nbr_idx[(long)k * D.kmax + t] = -1;
    Sol S;
    finish_ego(P, E, k, u, status, cnt, S);
    write_diag(P, E, S, k, pos, vel, D);
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
                                                         const double2* __restrict__ vel, cbf_diag D) {
    const int slot = blockIdx.x * kBlock + threadIdx.x;
    if (slot >= n) return;
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
                       diag_or_empty(diag));
    return (int)hipGetLastError();
}
