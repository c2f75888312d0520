// mc.hip -- batched Monte-Carlo rendezvous (SURVEY cfg5; meet_at_center.py:76-153 per scenario).
//
// One workgroup runs S = 256 / max(n_o, n_a) independent scenarios for all `steps` with the
// whole scenario state in LDS; thread k of a scenario owns obstacle k and agent k.  HBM is
// touched only to load the initial positions and to store the final ones + counters, so the
// kernel is FP64-VALU bound (cull + assembly + exact QP per agent per step).
#include "cbf_device.hpp"

using namespace cbf;


namespace {

// 3 waves per SIMD: the unrolled Seidel solve wants ~197 VGPRs (2 waves/SIMD); capped at 168 the
// compiler spills ~116 B per lane, and the third wave hides more than the spills cost: 1.62 ->
// 1.32 ms per 10 timesteps at 100 k scenarios (4 waves, 128 VGPRs and 272 B spilled: 1.93 ms;
// the rolled LDS solve at 101 VGPRs: 2.21 ms).  Bit-identical (tests/test_gpu_parity.py).
// ST: the statistics (violations, neighbour distances); without them (maxviol = NULL) the kernel
// computes none of them and writes the counters only.
template <bool FZ, bool ST>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 3))) k_mc_rollout(KP P, int n_scen, int n_o, int n_a, int steps, double T,
                                                       double rc, double rs, double so, double ga,
                                                       double2* __restrict__ pos, long long* __restrict__ counters,
                                                       double* __restrict__ maxviol, double* __restrict__ safety) {
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
    if (valid)
        for (int i = k; i < n; i += tps) sp[i] = pos[(long)scen * n + i];
    __syncthreads();
    long long c_calls = 0, c_relax = 0, c_box = 0, c_cap = 0;
    double mv = 0.0;       // max row violation over feasible (OPTIMAL) solves
    double mvo = 0.0;      // max violation of the original barrier rows over RELAXED solves
    double d2min = INFINITY;  // smallest distance^2 from an agent to a culled neighbour
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
            // cull pass: the exact test, hits compacted into a per-lane LDS list (reference
            // order: obstacles, then agents), then row assembly over those only
            int nh = 0;
            for (int j = 0; j < n; ++j) {
                const double2 pj = sp[j];
                double s;
                if (cull_keep(P, E.r0, E.r1, pj.x, pj.y, j < n_o, s)) {
                    if (nh < kHitCap) hit_lds[nh * kBlock + threadIdx.x] = j;
                    ++nh;
                    if (ST) d2min = pmin(d2min, s);
                }
            }
            if (nh <= kHitCap) {
                for (int i = 0; i < nh; ++i) {
                    const int j = hit_lds[i * kBlock + threadIdx.x];
                    const double2 pj = sp[j];
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
                const Sol Sl = solve_ego(P, E);
                clip_u(P, Sl, E, ux, uy);
                c_calls++;
                if (Sl.status == CBF_STATUS_RELAXED) c_relax++;
                if (Sl.status == CBF_STATUS_BOX_INFEASIBLE) c_box++;
                if (Sl.status == CBF_STATUS_RELAX_CAP) c_cap++;
                if (ST && Sl.status == CBF_STATUS_OPTIMAL) mv = Sl.viol > mv ? Sl.viol : mv;
                if (ST && Sl.status == CBF_STATUS_RELAXED) mvo = Sl.viol_orig > mvo ? Sl.viol_orig : mvo;
            }
        }
        __syncthreads();
        if (valid) {
            if (k < n_o) {
                const double2 p = sp[k], v = sv[k];
                const double2 q = make_double2(p.x + T * v.x, p.y + T * v.y);
                sp[k] = q;
            }
            if (k < n_a) {
                const double2 p = sp[n_o + k];
                const double2 q = make_double2(p.x + T * ux, p.y + T * uy);
                sp[n_o + k] = q;
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
    ml[3 * threadIdx.x] = mv;
    ml[3 * threadIdx.x + 1] = mvo;
    ml[3 * threadIdx.x + 2] = d2min;
    __syncthreads();
    if (valid && k == 0) {
        long long a = 0, b = 0, c = 0, d = 0;
        double m = 0.0, mo = 0.0, dm = INFINITY;
        for (int t = 0; t < tps; ++t) {
            const int th = ls * tps + t;
            a += cl[4 * th];
            b += cl[4 * th + 1];
            c += cl[4 * th + 2];
            d += cl[4 * th + 3];
            m = ml[3 * th] > m ? ml[3 * th] : m;
            mo = ml[3 * th + 1] > mo ? ml[3 * th + 1] : mo;
            dm = pmin(dm, ml[3 * th + 2]);
        }
        if (ST && safety) {
            safety[2l * scen] = mo;
            safety[2l * scen + 1] = dm;
        }
        counters[4l * scen + 0] = a;
        counters[4l * scen + 1] = b;
        counters[4l * scen + 2] = c;
        counters[4l * scen + 3] = d;
        if (ST) maxviol[scen] = m;
    }
}

}  // namespace

extern "C" int cbf_mc_rollout(const cbf_params* p, int32_t n_scen, int32_t n_o, int32_t n_a, int32_t steps,
                              double T, double rc, double rs, double so, double ga, double* pos, int64_t* counters,
                              double* maxviol, double* safety, void* stream) {
    if (!p || n_scen < 0 || n_o < 1 || n_a < 1 || n_o + n_a > kBlock || steps < 0) return CBF_EINVAL;
    if (n_scen == 0) return 0;
    if (!pos || !counters || (safety && !maxviol)) return CBF_EINVAL;
    const int tps = n_o > n_a ? n_o : n_a;
    const int S = kBlock / tps;
    const int stride = n_o + n_a + 1;
    // [positions | velocities | counter reduction (4 int64 + 3 double per thread)]
    const size_t lds = sizeof(double2) * (2 * S * stride) + (4 * sizeof(long long) + 3 * sizeof(double)) * kBlock;
    const int blocks = (n_scen + S - 1) / S;
    const auto kern = maxviol ? (p->f_is_zero ? k_mc_rollout<true, true> : k_mc_rollout<false, true>)
                              : (p->f_is_zero ? k_mc_rollout<true, false> : k_mc_rollout<false, false>);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), lds, (hipStream_t)stream, make_kp(p), n_scen, n_o,
                       n_a, steps, T, rc, rs, so, ga, reinterpret_cast<double2*>(pos),
                       reinterpret_cast<long long*>(counters), maxviol, safety);
    return (int)hipGetLastError();
}
