// rps.hip -- the robotarium (rps) pieces the reference scripts wrap around the filter, gfx950.
// SURVEY.md 8(f) rows 2-3 (third-party, absent from the image; parity unpinned):
//   uni_to_si_states / si_to_uni_dyn      cross_and_rescue.py:75,101,167; meet_at_center.py:61,80,148
//   Robotarium.set_velocities / step      cross_and_rescue.py:170,175;    meet_at_center.py:151,153
//   si_barrier_cert (with boundary)       cross_and_rescue.py:72,163;     meet_at_center.py:58,109
//
// The barrier certificate is a COUPLED QP over all 2N velocities of a scenario:
//   min |v - y|^2  s.t.  -2 e_ij.(v_i - v_j) <= gain h_ij^3   (every pair i < j)
//                        boundary rows per agent,
// y = the magnitude-thresholded input.  It is solved exactly by the Goldfarb-Idnani dual
// active-set method, one wavefront per scenario: lane l owns QP variable l (n = 2N <= 64), the
// factors J = L^-T Q (n x n) and R (q x q) live in LDS, rows are scanned 64 at a time, and each
// add / drop is a sequence of Givens rotations applied lane-parallel to J's rows.
#include "cbf_device.hpp"

using namespace cbf;

namespace {

constexpr int kCertMaxAgents = 32;  // n = 2N <= 64 = one lane per variable

struct CertArgs {
    double gain, gain_bnd, radius, mag;  // gain_bnd = 0.4 * gain (evaluated as rps does)
    double bx0, bx1, by0, by1;           // boundary_points
    double tol;                          // violation tolerance (relative to max(1, |b|))
    int max_iter;
};

// h^3 rounded once (np.power(h, 3) is libm pow): h^2 = p + e exactly, then p h + e h in one fma.
__device__ __forceinline__ double cube1(double h) {
    const double p = h * h;
    const double e = fma(h, h, -p);
    return fma(p, h, e * h);
}

// Reductions over the G lanes of one scenario's group (G divides the wave).
template <int G>
__device__ __forceinline__ void group_argmin(double& v, int& i) {
    for (int o = G / 2; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, G);
        const int oi = __shfl_xor(i, o, G);
        if (ov < v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

template <int G>
__device__ __forceinline__ double group_sum(double v) {
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

// LDS ordering between the lanes of the (single-wave) workgroup; groups of one wave run
// independent loops, so no workgroup barrier is used inside them.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pair index c (lexicographic i < j) -> (i, j).
__device__ __forceinline__ int2 pair_of(int c, int N) {
    int i = 0, off = 0;
    while (c >= off + (N - 1 - i)) {
        off += N - 1 - i;
        ++i;
    }
    return make_int2(i, i + 1 + (c - off));
}

// Row c of A applied to v (A c . v).  rij.y >= 0: pair (i, j); rij.y = -1 - kind: boundary row
// of agent rij.x, kind 0..3 = +y, -y, +x, -x (rps order).
__device__ __forceinline__ double row_dot(int2 ij, const double* xp, const double* v) {
    if (ij.y >= 0) {
        const double e0 = xp[2 * ij.x] - xp[2 * ij.y], e1 = xp[2 * ij.x + 1] - xp[2 * ij.y + 1];
        return (((-2.0 * e0) * v[2 * ij.x] + (-2.0 * e1) * v[2 * ij.x + 1]) + (2.0 * e0) * v[2 * ij.y]) +
               (2.0 * e1) * v[2 * ij.y + 1];
    }
    const int kind = -1 - ij.y;
    const double s = (kind & 1) ? -v[2 * ij.x + (kind < 2 ? 1 : 0)] : v[2 * ij.x + (kind < 2 ? 1 : 0)];
    return s;
}

// One scenario per group of G lanes (G >= 2N; 64 / G scenarios per wave), lane l of the group
// owns QP variable l; each group has its own LDS region of `sdw` doubles.
template <int G>
__global__ void __launch_bounds__(64) k_si_barrier_cert(CertArgs C, int N, int batch, long sdw,
                                                        const double2* __restrict__ dxi,
                                                        const double2* __restrict__ xs, double2* __restrict__ out,
                                                        int32_t* __restrict__ status, int32_t* __restrict__ iters,
                                                        int32_t* __restrict__ n_active) {
    extern __shared__ double lds_all[];
    const int n = 2 * N, m = N * (N - 1) / 2 + 4 * N, ld = n + 1;
    const int lane = threadIdx.x & (G - 1), grp = threadIdx.x / G;
    const long sc_raw = (long)blockIdx.x * (64 / G) + grp;
    const bool valid = sc_raw < batch;
    const long sc = valid ? sc_raw : batch - 1;  // idle groups shadow the last scenario, write nothing
    double* lds = lds_all + grp * sdw;
    double* J = lds;             // [n][ld]
    double* R = J + n * ld;      // [n][ld], column j = active constraint j
    double* brow = R + n * ld;   // [m]
    double* xp = brow + m;       // [n] agent positions (x-major per agent)
    double* xv = xp + n;         // [n] current iterate
    double* dv = xv + n;         // [n] d = J' n+
    double* rid = dv + n;        // [n] 1 / R[j][j]
    int2* rij = reinterpret_cast<int2*>(rid + n);  // [m]
    int* isact = reinterpret_cast<int*>(rij + m);  // [m]

    // inputs; magnitude threshold of rps (norms > magnitude_limit -> scaled onto the limit)
    double yl = 0.0;
    if (lane < N) {
        const double2 p = xs[sc * N + lane];
        xp[2 * lane] = p.x;
        xp[2 * lane + 1] = p.y;
    }
    {
        const int a = lane >> 1;
        if (lane < n) {
            const double2 d = dxi[sc * N + a];
            const double nrm = sqrt(d.x * d.x + d.y * d.y);
            double c = (lane & 1) ? d.y : d.x;
            if (nrm > C.mag) c *= C.mag / nrm;
            yl = c;
        }
    }
    for (int r = lane; r < n; r += G) {
        for (int c = 0; c < n; ++c) {
            J[r * ld + c] = (r == c) ? 1.0 / sqrt(2.0) : 0.0;
            R[r * ld + c] = 0.0;
        }
    }
    wave_sync();
    const int npair = N * (N - 1) / 2;
    for (int c = lane; c < m; c += G) {
        int2 ij;
        double b;
        if (c < npair) {
            ij = pair_of(c, N);
            const double e0 = xp[2 * ij.x] - xp[2 * ij.y], e1 = xp[2 * ij.x + 1] - xp[2 * ij.y + 1];
            const double h = (e0 * e0 + e1 * e1) - C.radius * C.radius;
            b = C.gain * cube1(h);
        } else {
            const int k = (c - npair) >> 2, kind = (c - npair) & 3;
            const double px = xp[2 * k], py = xp[2 * k + 1], r2 = C.radius / 2;
            double v;
            if (kind == 0) v = (C.by1 - r2) - py;
            else if (kind == 1) v = (-C.by0 - r2) + py;
            else if (kind == 2) v = (C.bx1 - r2) - px;
            else v = (-C.bx0 - r2) + px;
            b = C.gain_bnd * cube1(v);
            ij = make_int2(k, -1 - kind);
        }
        rij[c] = ij;
        brow[c] = b;
        isact[c] = 0;
    }
    double xl = yl;   // lane l: x_l
    double ul = 0.0;  // lane j < q: multiplier of active constraint j
    int actl = -1;    // lane j < q: its row
    int q = 0, st = CBF_CERT_MAXITER, it = 0;
    if (lane < n) xv[lane] = xl;
    wave_sync();

    while (true) {
        if (++it > C.max_iter) break;
        // most violated inactive row (first index on ties)
        double best = INFINITY;
        int bi = m;
        for (int c = lane; c < m; c += G) {
            if (isact[c]) continue;
            const double s = brow[c] - row_dot(rij[c], xp, xv);
            if (s < best) {
                best = s;
                bi = c;
            }
        }
        group_argmin<G>(best, bi);
        if (bi >= m || !(best < -C.tol * pmax(1.0, fabs(brow[bi])))) {
            st = CBF_CERT_OPTIMAL;
            break;
        }
        const int p = bi;
        const int2 pij = rij[p];
        // nonzeros of n+ = -A_p
        int k0, k1 = -1, k2 = -1, k3 = -1;
        double n0, n1 = 0.0, n2 = 0.0, n3 = 0.0;
        if (pij.y >= 0) {
            const double e0 = xp[2 * pij.x] - xp[2 * pij.y], e1 = xp[2 * pij.x + 1] - xp[2 * pij.y + 1];
            k0 = 2 * pij.x, k1 = k0 + 1, k2 = 2 * pij.y, k3 = k2 + 1;
            n0 = 2.0 * e0, n1 = 2.0 * e1, n2 = -2.0 * e0, n3 = -2.0 * e1;
        } else {
            const int kind = -1 - pij.y;
            k0 = 2 * pij.x + (kind < 2 ? 1 : 0);
            n0 = (kind & 1) ? 1.0 : -1.0;
        }
        double up = 0.0;
        bool infeasible = false;
        while (true) {
            // d = J' n+ (lane = column)
            double dl = 0.0;
            if (lane < n) {
                dl = n0 * J[k0 * ld + lane];
                if (k1 >= 0) dl = ((dl + n1 * J[k1 * ld + lane]) + n2 * J[k2 * ld + lane]) + n3 * J[k3 * ld + lane];
                dv[lane] = dl;
            }
            wave_sync();
            // z = J[:, q:] d[q:] (lane = row)
            // (four partial sums: the LDS loads of consecutive columns overlap)
            double zl = 0.0;
            if (lane < n) {
                double z0 = 0.0, z1 = 0.0, z2 = 0.0, z3 = 0.0;
                const double* Jr = J + lane * ld;
                int c = q;
                for (; c + 4 <= n; c += 4) {
                    z0 += Jr[c] * dv[c];
                    z1 += Jr[c + 1] * dv[c + 1];
                    z2 += Jr[c + 2] * dv[c + 2];
                    z3 += Jr[c + 3] * dv[c + 3];
                }
                for (; c < n; ++c) z0 += Jr[c] * dv[c];
                zl = (z0 + z1) + (z2 + z3);
            }
            // r = R^-1 d[:q], column-oriented back substitution (lane j ends with r_j); rid holds
            // the reciprocals of R's diagonal
            double rl = lane < q ? dl : 0.0;
            for (int j = q - 1; j >= 0; --j) {
                const double rj = __shfl(rl, j, G) * rid[j];
                if (lane == j) rl = rj;
                else if (lane < j) rl -= R[lane * ld + j] * rj;
            }
            // partial (dual) step: the first active constraint whose multiplier reaches 0
            double t1 = INFINITY;
            int kk = G;
            if (lane < q && rl > 0.0) {
                t1 = ul / rl;
                kk = lane;
            }
            group_argmin<G>(t1, kk);
            const double zn = group_sum<G>((lane >= q && lane < n) ? dl * dl : 0.0);
            const double dd = group_sum<G>(lane < n ? dl * dl : 0.0);
            double t2 = INFINITY;
            if (zn > 1e-28 * dd) t2 = -(brow[p] - row_dot(pij, xp, xv)) / zn;
            if (t1 == INFINITY && t2 == INFINITY) {
                infeasible = true;
                break;
            }
            const bool full = t2 <= t1;
            const double t = full ? t2 : t1;
            if (t2 != INFINITY) {
                xl += t * zl;
                if (lane < n) xv[lane] = xl;
            }
            if (lane < q) ul -= t * rl;
            up += t;
            if (full) {
                // add p: one Householder reflection H = I - v v' / (sg vq) maps d[q:] onto
                // -sg e_q (v = d[q:] + sg e_q, sg = |d[q:]| with the sign of d_q); J[:, q:] <- J[:, q:] H,
                // lane-parallel over J's rows
                const double dq = __shfl(dl, q, G);
                const double sg = copysign(sqrt(zn), dq);
                const double vq = dq + sg;
                const double beta = 1.0 / (sg * vq);
                if (lane < n) {
                    double* Jr = J + lane * ld;
                    double a0 = Jr[q] * vq, a1 = 0.0, a2 = 0.0, a3 = 0.0;
                    int c = q + 1;
                    for (; c + 3 <= n; c += 3) {
                        a1 += Jr[c] * dv[c];
                        a2 += Jr[c + 1] * dv[c + 1];
                        a3 += Jr[c + 2] * dv[c + 2];
                    }
                    for (; c < n; ++c) a1 += Jr[c] * dv[c];
                    const double f = beta * ((a0 + a1) + (a2 + a3));
                    Jr[q] -= f * vq;
                    for (c = q + 1; c < n; ++c) Jr[c] -= f * dv[c];
                }
                const double carry = -sg;
                if (lane < q) R[lane * ld + q] = dl;
                if (lane == q) {
                    R[q * ld + q] = carry;
                    rid[q] = 1.0 / carry;
                    ul = up;
                    actl = p;
                    isact[p] = 1;
                }
                ++q;
                wave_sync();
                break;
            }
            // drop active constraint kk: delete R's column kk, restore the triangle with Givens on
            // rows (j, j+1), the same rotations on J's columns (j, j+1)
            if (lane < q) {
                for (int j = kk; j < q - 1; ++j) R[lane * ld + j] = R[lane * ld + j + 1];
                R[lane * ld + q - 1] = 0.0;
            }
            wave_sync();
            if (lane >= kk && lane < q - 1) rid[lane] = 1.0 / R[lane * ld + lane];  // shifted diagonal
            wave_sync();
            for (int j = kk; j < q - 1; ++j) {
                const double a = R[j * ld + j], b = R[(j + 1) * ld + j];
                const double h = hypot(a, b);
                wave_sync();
                if (h != 0.0) {
                    const double cs = a / h, sn = b / h;
                    if (lane >= j && lane < q - 1) {
                        const double Ra = R[j * ld + lane], Rb = R[(j + 1) * ld + lane];
                        const double Rn = cs * Ra + sn * Rb;
                        R[j * ld + lane] = Rn;
                        R[(j + 1) * ld + lane] = lane == j ? 0.0 : -sn * Ra + cs * Rb;
                        if (lane == j) rid[j] = 1.0 / Rn;
                    }
                    if (lane < n) {
                        const double Ja = J[lane * ld + j], Jb = J[lane * ld + j + 1];
                        J[lane * ld + j] = cs * Ja + sn * Jb;
                        J[lane * ld + j + 1] = -sn * Ja + cs * Jb;
                    }
                }
                wave_sync();
            }
            const int gone = __shfl(actl, kk, G);
            const double un = __shfl_down(ul, 1, G);
            const int an = __shfl_down(actl, 1, G);
            if (lane >= kk && lane < q - 1) {
                ul = un;
                actl = an;
            }
            if (lane == q - 1) {
                ul = 0.0;
                actl = -1;
            }
            if (lane == 0) isact[gone] = 0;
            --q;
            wave_sync();
        }
        if (infeasible) {
            st = CBF_CERT_INFEASIBLE;
            break;
        }
    }
    const double val = st == CBF_CERT_OPTIMAL ? xl : yl;
    const double ox = __shfl(val, (2 * lane) & (G - 1), G), oy = __shfl(val, (2 * lane + 1) & (G - 1), G);
    if (valid && lane < N) out[sc * N + lane] = make_double2(ox, oy);
    if (valid && lane == 0) {
        status[sc] = st;
        if (iters) iters[sc] = it;
        if (n_active) n_active[sc] = q;
    }
}

struct UniArgs {
    double l, inv_l, wlim;             // projection distance, 1 / l, angular velocity limit
    double vmax, wmax;                 // set_velocities saturation
    double c_dd, c_v, c_w, lb, wheel;  // 1/(2r), r/2, r/l, base length, max wheel speed
    double dt;
    int wheel_threshold;
};

__global__ void __launch_bounds__(kBlock) k_uni_to_si(UniArgs U, int n, const double* __restrict__ poses,
                                                     double2* __restrict__ si) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double x = poses[3 * i], y = poses[3 * i + 1], th = poses[3 * i + 2];
    si[i] = make_double2(x + U.l * cos(th), y + U.l * sin(th));
}

__device__ __forceinline__ double sgn(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : v); }

// MODE 0: si_to_uni_dyn -> set_velocities -> Robotarium.step (motor threshold, Euler, atan2
// wrap); MODE 1: si_to_uni_dyn alone (dxi -> dxu); MODE 2: set_velocities + step from dxu.
// Every expression keeps the order the numpy source evaluates it in.
template <int MODE>
__global__ void __launch_bounds__(kBlock) k_unicycle(UniArgs U, int n, double* __restrict__ poses,
                                                    const double2* __restrict__ in, double2* __restrict__ dxu_out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double x = poses[3 * i], y = poses[3 * i + 1], th = poses[3 * i + 2];
    const double2 d = in[i];
    const double cs = cos(th), ss = sin(th);
    double v, w;
    if (MODE != 2) {
        v = cs * d.x + ss * d.y;  // si_to_uni_dyn
        w = U.inv_l * (-ss * d.x + cs * d.y);
        if (w > U.wlim) w = U.wlim;
        if (w < -U.wlim) w = -U.wlim;
        if (dxu_out) dxu_out[i] = make_double2(v, w);
        if (MODE == 1) return;
    } else {
        v = d.x;
        w = d.y;
    }
    if (fabs(v) > U.vmax) v = U.vmax * sgn(v);  // set_velocities
    if (fabs(w) > U.wmax) w = U.wmax * sgn(w);
    if (U.wheel_threshold) {                    // step(): _uni_to_diff, clamp, _diff_to_uni
        double wl = U.c_dd * (2.0 * v - U.lb * w), wr = U.c_dd * (2.0 * v + U.lb * w);
        if (fabs(wl) > U.wheel) wl = U.wheel * sgn(wl);
        if (fabs(wr) > U.wheel) wr = U.wheel * sgn(wr);
        v = U.c_v * (wl + wr);
        w = U.c_w * (wr - wl);
    }
    poses[3 * i] = x + (U.dt * cs) * v;
    poses[3 * i + 1] = y + (U.dt * ss) * v;
    const double t2 = th + U.dt * w;
    poses[3 * i + 2] = atan2(sin(t2), cos(t2));
}

inline int nblk(long n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

extern "C" int cbf_cert_params_init(cbf_cert_params* c, double barrier_gain, double safety_radius,
                                    double magnitude_limit, const double* boundary_points4) {
    if (!c) return CBF_EINVAL;
    c->barrier_gain = barrier_gain;
    c->safety_radius = safety_radius;
    c->magnitude_limit = magnitude_limit;
    const double bp[4] = {-1.6, 1.6, -1.0, 1.0};
    for (int i = 0; i < 4; ++i) c->boundary_points[i] = boundary_points4 ? boundary_points4[i] : bp[i];
    c->viol_tol = 1e-12;
    c->max_iter = 0;
    return 0;
}

extern "C" size_t cbf_si_barrier_cert_lds_bytes(int32_t n_agents) {
    if (n_agents < 1 || n_agents > kCertMaxAgents) return 0;
    const size_t n = 2 * (size_t)n_agents, m = (size_t)n_agents * (n_agents - 1) / 2 + 4 * (size_t)n_agents;
    return 8 * (2 * n * (n + 1) + m + 4 * n) + 8 * m + 4 * m;
}

extern "C" int cbf_si_barrier_cert(const cbf_cert_params* c, int32_t batch, int32_t n_agents, const double* dxi,
                                   const double* x, double* out, int32_t* status, int32_t* iters, int32_t* n_active,
                                   void* stream) {
    if (!c || batch < 0 || n_agents < 1 || n_agents > kCertMaxAgents) return CBF_EINVAL;
    if (batch == 0) return 0;
    if (!dxi || !x || !out || !status) return CBF_EINVAL;
    CertArgs A;
    A.gain = c->barrier_gain;
    A.gain_bnd = 0.4 * c->barrier_gain;
    A.radius = c->safety_radius;
    A.mag = c->magnitude_limit;
    A.bx0 = c->boundary_points[0];
    A.bx1 = c->boundary_points[1];
    A.by0 = c->boundary_points[2];
    A.by1 = c->boundary_points[3];
    A.tol = c->viol_tol;
    const int m = n_agents * (n_agents - 1) / 2 + 4 * n_agents;
    A.max_iter = c->max_iter > 0 ? c->max_iter : 10 * (m + 2 * n_agents) + 10;
    // per-scenario LDS region, rounded to 16 B.  Small scenarios share a wave: groups of G = 8 / 16
    // lanes (G >= 2N) for N <= 8; beyond that one scenario per wave (2 per wave measured slower
    // at N = 16: the doubled LDS per workgroup costs more resident waves than it saves lanes)
    const size_t per = (cbf_si_barrier_cert_lds_bytes(n_agents) + 15) / 16 * 16;
    const int G = 2 * n_agents <= 8 ? 8 : (2 * n_agents <= 16 ? 16 : 64);
    const int spw = 64 / G;
    const int blocks = (batch + spw - 1) / spw;
    auto kern = G == 8 ? k_si_barrier_cert<8> : (G == 16 ? k_si_barrier_cert<16> : k_si_barrier_cert<64>);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), per * spw, (hipStream_t)stream, A, n_agents, batch,
                       (long)(per / 8), reinterpret_cast<const double2*>(dxi), reinterpret_cast<const double2*>(x),
                       reinterpret_cast<double2*>(out), status, iters, n_active);
    return (int)hipGetLastError();
}

static UniArgs make_uni(const cbf_unicycle_params* u) {
    UniArgs U;
    U.l = u->projection_distance;
    U.inv_l = 1 / u->projection_distance;
    U.wlim = u->angular_velocity_limit;
    U.vmax = u->max_linear_velocity;
    U.wmax = u->max_angular_velocity;
    U.c_dd = 1 / (2 * u->wheel_radius);
    U.c_v = u->wheel_radius / 2;
    U.c_w = u->wheel_radius / u->base_length;
    U.lb = u->base_length;
    U.wheel = u->max_wheel_velocity;
    U.dt = u->time_step;
    U.wheel_threshold = u->wheel_threshold;
    return U;
}

extern "C" int cbf_unicycle_params_init(cbf_unicycle_params* u) {
    if (!u) return CBF_EINVAL;
    u->projection_distance = 0.05;
    u->angular_velocity_limit = M_PI;
    u->time_step = 0.033;
    u->wheel_radius = 0.016;
    u->base_length = 0.105;
    u->max_linear_velocity = 0.2;
    const double robot_diameter = 0.11;
    u->max_angular_velocity = 2 * (u->wheel_radius / robot_diameter) * (u->max_linear_velocity / u->wheel_radius);
    u->max_wheel_velocity = u->max_linear_velocity / u->wheel_radius;
    u->wheel_threshold = 1;
    return 0;
}

extern "C" int cbf_uni_to_si(const cbf_unicycle_params* u, int32_t n, const double* poses, double* si,
                             void* stream) {
    if (!u || n < 0 || !(u->projection_distance != 0)) return CBF_EINVAL;
    if (n == 0) return 0;
    if (!poses || !si) return CBF_EINVAL;
    hipLaunchKernelGGL(k_uni_to_si, dim3(nblk(n)), dim3(kBlock), 0, (hipStream_t)stream, make_uni(u), n, poses,
                       reinterpret_cast<double2*>(si));
    return (int)hipGetLastError();
}

extern "C" int cbf_unicycle_advance(const cbf_unicycle_params* u, int32_t n, double* poses, const double* dxi,
                                    double* dxu, int32_t mode, void* stream) {
    if (!u || n < 0 || mode < 0 || mode > 2 || !(u->projection_distance != 0) || !(u->base_length != 0) ||
        !(u->wheel_radius != 0))
        return CBF_EINVAL;
    if (n == 0) return 0;
    if (!poses || !dxi || (mode == 1 && !dxu)) return CBF_EINVAL;
    auto k = mode == 0 ? k_unicycle<0> : (mode == 1 ? k_unicycle<1> : k_unicycle<2>);
    hipLaunchKernelGGL(k, dim3(nblk(n)), dim3(kBlock), 0, (hipStream_t)stream, make_uni(u), n, poses,
                       reinterpret_cast<const double2*>(dxi), reinterpret_cast<double2*>(dxu));
    return (int)hipGetLastError();
}
