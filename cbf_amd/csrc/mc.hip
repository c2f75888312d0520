// mc.hip -- batched Monte-Carlo rendezvous (SURVEY cfg5; meet_at_center.py:76-153 per scenario).
//
// One workgroup runs S = 256 / max(n_o, n_a) independent scenarios for all `steps` with the
// whole scenario state in LDS; thread k of a scenario owns obstacle k and agent k.  HBM is
// touched only to load the initial positions and to store the final ones + counters, so the
// kernel is FP64-VALU bound (cull + assembly + exact QP per agent per step).
#include "cbf_device.hpp"

using namespace cbf;

// tools/ablate.py switches: fp32 cull screen, solve_easy fast path
#ifndef CBF_MC_SCREEN
#define CBF_MC_SCREEN 0
#endif
#ifndef CBF_MC_EASY
#define CBF_MC_EASY 0
#endif

namespace {

template <bool FZ>
__global__ void __launch_bounds__(kBlock) k_mc_rollout(KP P, int n_scen, int n_o, int n_a, int steps, double T,
                                                       double rc, double rs, double so, double ga,
                                                       double2* __restrict__ pos, long long* __restrict__ counters,
                                                       double* __restrict__ maxviol) {
    extern __shared__ double2 lds[];
    __shared__ int hit_lds[kHitCap * kBlock];
    const int tps = n_o > n_a ? n_o : n_a;
    const int S = kBlock / tps;
    const int n = n_o + n_a;
    const int stride = n + 1;  // +1 entry of padding: scenarios start on different LDS banks
    const int ls = threadIdx.x / tps, k = threadIdx.x % tps;
    const int scen = blockIdx.x * S + ls;
    const bool valid = ls < S && scen < n_scen;
    double2* sp = lds + (valid ? ls : 0) * stride;
    double2* sv = lds + S * stride + (valid ? ls : 0) * stride;
    // fp32 copies of the positions for the cull screen, after the counter-reduction area
    float2* sp32 = reinterpret_cast<float2*>(lds + 2 * S * stride + kBlock * 3) + (valid ? ls : 0) * stride;
    if (valid)
        for (int i = k; i < n; i += tps) {
            const double2 p = pos[(long)scen * n + i];
            sp[i] = p;
            sp32[i] = make_float2((float)p.x, (float)p.y);
        }
    __syncthreads();
    long long c_calls = 0, c_relax = 0, c_box = 0, c_cap = 0;
    double mv = 0.0;
    for (int step = 0; step < steps; ++step) {
        if (valid) {
            if (k < n_o) {  // cyclic pursuit: ring neighbour k+1, rotated, scaled
                const double2 xi = sp[k], xj = sp[k + 1 < n_o ? k + 1 : 0];
                const double a0 = 0.0 + (xj.x - xi.x), a1 = 0.0 + (xj.y - xi.y);
                const double v0 = fma(a1, -rs, a0 * rc), v1 = fma(a1, rc, a0 * rs);
                sv[k] = make_double2(v0 * so, v1 * so);
            }
            if (k < n_a) {  // complete-graph consensus over the free agents
                const double2 xi = sp[n_o + k];
                double a0 = 0.0, a1 = 0.0;
                for (int j = 0; j < n_a; ++j) {
                    if (j == k) continue;
                    const double2 xj = sp[n_o + j];
                    a0 = a0 + (xj.x - xi.x);
                    a1 = a1 + (xj.y - xi.y);
                }
                sv[n_o + k] = make_double2(a0 * ga, a1 * ga);
            }
        }
        __syncthreads();
        double ux = 0.0, uy = 0.0;
        if (valid && k < n_a) {
            const double2 pe = sp[n_o + k], ve = sv[n_o + k];
            Ego E;
            ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
            // cull pass: an fp32 screen (conservative: screen_threshold) over the fp32 copies,
            // candidates it lets through compacted into a per-lane LDS list, then the exact fp64
            // cull test + assembly over those only
            int nh = 0;
#if CBF_MC_SCREEN
            const float t32 = screen_threshold(P.cull_t, pmax(fabs(E.r0), fabs(E.r1)) + sqrt(P.cull_t));
            if (t32 > 0.0f) {
                const float ex = (float)E.r0, ey = (float)E.r1;
                for (int j = 0; j < n; ++j) {
                    const float2 c = sp32[j];
                    const float d0 = c.x - ex, d1 = c.y - ey;
                    if (__builtin_fmaf(d0, d0, d1 * d1) < t32) {
                        if (nh < kHitCap) hit_lds[nh * kBlock + threadIdx.x] = j;
                        ++nh;
                    }
                }
            } else {
                nh = kHitCap + 1;  // screen off (non-finite or huge coordinates): the direct path
            }
#else
            for (int j = 0; j < n; ++j) {
                const double2 pj = sp[j];
                double s;
                if (cull_keep(P, E.r0, E.r1, pj.x, pj.y, j < n_o, s)) {
                    if (nh < kHitCap) hit_lds[nh * kBlock + threadIdx.x] = j;
                    ++nh;
                }
            }
#endif
            if (nh <= kHitCap) {
                for (int i = 0; i < nh; ++i) {
                    const int j = hit_lds[i * kBlock + threadIdx.x];
                    const double2 pj = sp[j];
#if CBF_MC_SCREEN
                    double s;
                    if (!cull_keep(P, E.r0, E.r1, pj.x, pj.y, j < n_o, s)) continue;
#endif
                    const double2 vj = sv[j];
                    ego_add<FZ>(P, E, pj.x, pj.y, vj.x, vj.y);
                }
            } else {
                for (int j = 0; j < n; ++j) {
                    const double2 pj = sp[j];
                    double s;
                    if (cull_keep(P, E.r0, E.r1, pj.x, pj.y, j < n_o, s)) {
                        const double2 vj = sv[j];
                        ego_add<FZ>(P, E, pj.x, pj.y, vj.x, vj.y);
                    }
                }
            }
            if (E.count == 0) {
                ux = E.u0x;
                uy = E.u0y;
            } else {
#if CBF_MC_EASY
                Sol Sl;
                if (!solve_easy(P, E, Sl)) Sl = solve_ego(P, E);  // bit-identical on the easy path
#else
                const Sol Sl = solve_ego(P, E);
#endif
                clip_u(P, Sl, E, ux, uy);
                c_calls++;
                if (Sl.status == CBF_STATUS_RELAXED) c_relax++;
                if (Sl.status == CBF_STATUS_BOX_INFEASIBLE) c_box++;
                if (Sl.status == CBF_STATUS_RELAX_CAP) c_cap++;
                if (Sl.status == CBF_STATUS_OPTIMAL || Sl.status == CBF_STATUS_RELAXED) mv = Sl.viol > mv ? Sl.viol : mv;
            }
        }
        __syncthreads();
        if (valid) {
            if (k < n_o) {
                const double2 p = sp[k], v = sv[k];
                const double2 q = make_double2(p.x + T * v.x, p.y + T * v.y);
                sp[k] = q;
                sp32[k] = make_float2((float)q.x, (float)q.y);
            }
            if (k < n_a) {
                const double2 p = sp[n_o + k];
                const double2 q = make_double2(p.x + T * ux, p.y + T * uy);
                sp[n_o + k] = q;
                sp32[n_o + k] = make_float2((float)q.x, (float)q.y);
            }
        }
        __syncthreads();
    }
    if (valid)
        for (int i = k; i < n; i += tps) pos[(long)scen * n + i] = sp[i];
    // per-scenario counter reduction through LDS (the velocity area is free now)
    long long* cl = reinterpret_cast<long long*>(lds + 2 * S * stride);
    double* ml = reinterpret_cast<double*>(cl + 4 * kBlock);
    cl[4 * threadIdx.x + 0] = c_calls;
    cl[4 * threadIdx.x + 1] = c_relax;
    cl[4 * threadIdx.x + 2] = c_box;
    cl[4 * threadIdx.x + 3] = c_cap;
    ml[threadIdx.x] = mv;
    __syncthreads();
    if (valid && k == 0) {
        long long a = 0, b = 0, c = 0, d = 0;
        double m = 0.0;
        for (int t = 0; t < tps; ++t) {
            const int th = ls * tps + t;
            a += cl[4 * th];
            b += cl[4 * th + 1];
            c += cl[4 * th + 2];
            d += cl[4 * th + 3];
            m = ml[th] > m ? ml[th] : m;
        }
        counters[4l * scen + 0] = a;
        counters[4l * scen + 1] = b;
        counters[4l * scen + 2] = c;
        counters[4l * scen + 3] = d;
        maxviol[scen] = m;
    }
}

}  // namespace

extern "C" int cbf_mc_rollout(const cbf_params* p, int32_t n_scen, int32_t n_o, int32_t n_a, int32_t steps,
                              double T, double rc, double rs, double so, double ga, double* pos, int64_t* counters,
                              double* maxviol, void* stream) {
    if (!p || n_scen < 0 || n_o < 1 || n_a < 1 || n_o + n_a > kBlock || steps < 0) return CBF_EINVAL;
    if (n_scen == 0) return 0;
    if (!pos || !counters || !maxviol) return CBF_EINVAL;
    const int tps = n_o > n_a ? n_o : n_a;
    const int S = kBlock / tps;
    const int stride = n_o + n_a + 1;
    // [positions | velocities | counter reduction (3 double2 per thread) | fp32 positions]
    const size_t lds = sizeof(double2) * (2 * S * stride + 3 * kBlock) + sizeof(float2) * S * stride;
    const int blocks = (n_scen + S - 1) / S;
    hipLaunchKernelGGL(p->f_is_zero ? k_mc_rollout<true> : k_mc_rollout<false>, dim3(blocks), dim3(kBlock), lds, (hipStream_t)stream, make_kp(p), n_scen, n_o,
                       n_a, steps, T, rc, rs, so, ga, reinterpret_cast<double2*>(pos),
                       reinterpret_cast<long long*>(counters), maxviol);
    return (int)hipGetLastError();
}
