// cbf_device.hpp -- device-side building blocks of the CBF safety filter (gfx950).
//
// Everything here is IEEE fp64 with no contraction (built with -ffp-contract=off); the only
// fused multiply-adds are the explicit fma() calls that reproduce the evaluation order numpy
// uses in the reference (probed, pinned by tests/golden):
//   hs_p @ d, np.dot(hs_p, g@u0)  -> fma chain     (cbf.py:55-59)
//   g @ u0                        -> fma(g[r,0], u0x, g[r,1]*u0y)
//   f @ d                         -> (f0 d0 + f2 d2) + (f1 d1 + f3 d3) per row (cbf.py:55)
//   v @ rotation                  -> fma(v1, R[1,c], v0*R[0,c])  (cross_and_rescue.py:118)
// so that results are bit-identical to the CPU oracle (oracle/cbf_oracle.c).  BLAS accumulates
// into a zeroed output, so numpy never returns -0.0 from these products; of them only the
// quadrant term c can carry a zero's sign into a barrier rhs b = (gamma (H - dmin) + L_f) + c
// (once c is +0 or nonzero, the other terms' zero signs cannot reach b), so only c is
// canonicalised (0.0 + c) here.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "cbf_amd.h"

#ifndef CBF_FLUSH_U
#define CBF_FLUSH_U 4
#endif
#ifndef CBF_SCAN_U
#define CBF_SCAN_U 6
#endif
static_assert(CBF_FLUSH_U >= 1 && CBF_SCAN_U >= 1, "loads in flight per lane");
namespace cbf {

constexpr double FEAS_TOL = 1e-12;
constexpr double ACTIVE_TOL = 1e-12;
constexpr int kBlock = 256;

// Kernel-argument copy of cbf_params (passed by value: lives in the kernarg segment / SGPRs).
struct KP {
    double ms, dmin, k, gamma;
    double f[16];
    double g[8];
    double cull_t;
    double n0[4], n1[4];  // quadrant normals L_g (host-computed with the reference's order)
    double z[4];          // n0[q] * 0.0 + n1[q] * 0.0: the CBF planes' a.x at the origin (solve_fast)
    int f_zero;
    int relax_cap;
    // window cull (CBF_RUN_WINDOW_CULL): the smallest double d with d * d >= cull_t, so that a
    // coordinate difference e with |e| > d makes e * e >= cull_t (rounding is monotone), i.e. the
    // candidate cannot pass the cull test s < cull_t of cross_and_rescue.py:141-150
    double win_d;
    double win_dn;  // nextafter(win_d, +inf): x - y >= win_dn in real arithmetic proves fl(x - y) > win_d
};

inline KP make_kp(const cbf_params* p) {
    KP k;
    k.ms = p->max_speed;
    k.dmin = p->dmin;
    k.k = p->k;
    k.gamma = p->gamma;
    for (int i = 0; i < 16; ++i) k.f[i] = p->f[i];
    for (int i = 0; i < 8; ++i) k.g[i] = p->g[i];
    k.cull_t = p->cull_t;
    for (int q = 0; q < 4; ++q) {
        k.n0[q] = p->nrm[q][0];
        k.n1[q] = p->nrm[q][1];
        k.z[q] = k.n0[q] * 0.0 + k.n1[q] * 0.0;
    }
    k.f_zero = p->f_is_zero;
    k.relax_cap = p->relax_cap;
    double d = sqrt(p->cull_t > 0 ? p->cull_t : 0.0);
    while (d * d < p->cull_t) d = nextafter(d, INFINITY);
    k.win_d = d;
    k.win_dn = nextafter(d, INFINITY);
    return k;
}

#ifndef CBF_NT_STORES
#define CBF_NT_STORES 0
#endif
// a streaming 16-B output store (non-temporal with CBF_NT_STORES: written through rather than left
// dirty in L2 for the kernel's end)
__device__ __forceinline__ void st_stream(double2* p, double2 v) {
#if CBF_NT_STORES
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
#else
    *p = v;
#endif
}
__device__ __forceinline__ double pmin(double a, double b) { return (b < a) ? b : a; }  // Python min(a, b)
__device__ __forceinline__ double pmax(double a, double b) { return (b > a) ? b : a; }  // Python max(a, b)
// v_min_f64 (volatile: kept under its branch, not speculated into a select).  For the per-quadrant
// minima of barrier rows g it equals `g < m ? g : m` (m the running minimum, never NaN): g is never
// -0 (H - dmin of a hit is +0 at worst, and L_f only adds to it) nor a signalling NaN (arithmetic
// results), and IEEE-mode min returns m for a quiet-NaN g, as the compare skips it.
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// pmax(1.0, fabs(b)) as one v_max_f64 (the compiler's form canonicalises |b| first: two
// instructions).  The same value for every b the solvers see: arithmetic results, so never a
// signalling NaN, and IEEE-mode max returns 1.0 for a quiet NaN as the compare-select does.
__device__ __forceinline__ double max1abs(double b) {
    double r;
    asm("v_max_f64 %0, 1.0, |%1|" : "=v"(r) : "v"(b));
    return r;
}

// fp32 screen of the cull test.  A candidate can pass the exact fp64 test s = e0^2 + e1^2 < cull_t
// (cross_and_rescue.py:141-150) only if S = the fp32 distance^2 of the fp32-rounded coordinates
// is below the returned T32; the screen only rejects, every candidate it lets through is
// re-tested exactly.  Bound: with |coords| <= M, u = 2^-24, |E_k - e_k| <= eta = 2uM + u(r + 2uM)
// (+ fp64 and subnormal slack) for |e_k| < r = sqrt(cull_t), so S <= (cull_t + 2 sqrt2 r eta +
// 2 eta^2)(1 + 3u); T32 adds slack on every term and rounds up.  M beyond 1e30 (or NaN) switches
// the screen off (returns -1).  For a true neighbour both coordinates lie within r of the ego's,
// so M = max(|ego coords|) + r suffices.
__device__ __forceinline__ float screen_threshold(double cull_t, double M) {
    if (!(M <= 1e30)) return -1.0f;
    const double u = 0x1p-24;
    const double r = sqrt(cull_t) * (1.0 + 1e-12);
    const double eta = 2.0 * u * M + u * (r + 2.0 * u * M) + 1e-14 * r + 1e-35;
    const double T = (cull_t * (1.0 + 1e-12) + 3.0 * r * eta + 3.0 * eta * eta) * (1.0 + 8.0 * u);
    float t32 = (float)T;
    if ((double)t32 < T) t32 = __uint_as_float(__float_as_uint(t32) + 1u);  // next float up (T > 0)
    return t32;
}

// One ego's accumulated QP: its state, g@u0, and the per-sign-quadrant minimum barrier rhs.
struct Ego {
    double r0, r1, r2, r3;  // robot_state (x, y, vx, vy)
    double u0x, u0y;        // nominal control
    double gu0, gu1, gu2, gu3;
    double bq0, bq1, bq2, bq3;
    unsigned present;  // bit q: quadrant q has >= 1 neighbour
    int count;         // neighbours
};

__device__ __forceinline__ void ego_init(const KP& P, Ego& E, double px, double py, double vx, double vy, double ux,
                                         double uy) {
    E.r0 = px;
    E.r1 = py;
    E.r2 = vx;
    E.r3 = vy;
    E.u0x = ux;
    E.u0y = uy;
    E.gu0 = fma(P.g[0], ux, P.g[1] * uy);
    E.gu1 = fma(P.g[2], ux, P.g[3] * uy);
    E.gu2 = fma(P.g[4], ux, P.g[5] * uy);
    E.gu3 = fma(P.g[6], ux, P.g[7] * uy);
    E.bq0 = E.bq1 = E.bq2 = E.bq3 = INFINITY;
    E.present = 0u;
    E.count = 0;
}

// L_f = hs_p @ (f @ d) (cbf.py:55): numpy's dgemv_t row order, then the hs_p fma chain.
__device__ __forceinline__ double lf_term(const KP& P, double d0, double d1, double d2, double d3, double sx,
                                         double sy, double ksx, double ksy) {
    double fd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        fd[i] = (P.f[4 * i] * d0 + P.f[4 * i + 2] * d2) + (P.f[4 * i + 1] * d1 + P.f[4 * i + 3] * d3);
    return fma(ksy, fd[3], fma(ksx, fd[2], fma(sy, fd[1], sx * fd[0])));
}

// Barrier row rhs for neighbour o (cbf.py:38-59); q = sign quadrant (cbf.py:47-53, -0.0 -> +1).
// FZ: compile-time "f == 0" (the callers' dynamics, cross_and_rescue.py:31) -> L_f = 0 with f
// never read; otherwise the runtime flag decides.
template <bool FZ = false>
__device__ __forceinline__ double row_b(const KP& P, const Ego& E, double o0, double o1, double o2, double o3,
                                        int& q) {
    const double d0 = E.r0 - o0, d1 = E.r1 - o1, d2 = E.r2 - o2, d3 = E.r3 - o3;
    const bool nx = d0 < 0, ny = d1 < 0;
    const double sx = nx ? -1.0 : 1.0, sy = ny ? -1.0 : 1.0;
    const double ksx = P.k * sx, ksy = P.k * sy;
    const double H = fma(ksy, d3, fma(ksx, d2, fma(sy, d1, sx * d0)));
    double Lf = 0.0;
    if (!FZ && !P.f_zero) Lf = lf_term(P, d0, d1, d2, d3, sx, sy, ksx, ksy);
    const double c = 0.0 + fma(ksy, E.gu3, fma(ksx, E.gu2, fma(sy, E.gu1, sx * E.gu0)));
    q = (nx ? 1 : 0) | (ny ? 2 : 0);
    // with f == 0 the reference adds L_f = +-0, which leaves every nonzero value unchanged
    // (only the sign of an exactly-zero sum can differ); the compile-time path drops the add
    if (FZ) return P.gamma * (H - P.dmin) + c;
    return (P.gamma * (H - P.dmin) + Lf) + c;
}

// row_b's quadrant term c (the g(x) u0 part of cbf.py:55-59) for sign quadrant q, same expression.
__device__ __forceinline__ double quad_c(const KP& P, const Ego& E, int q) {
    const double sx = (q & 1) ? -1.0 : 1.0, sy = (q & 2) ? -1.0 : 1.0;
    const double ksx = P.k * sx, ksy = P.k * sy;
    return 0.0 + fma(ksy, E.gu3, fma(ksx, E.gu2, fma(sy, E.gu1, sx * E.gu0)));
}

// row_b without the quadrant term c, for a neighbour whose position differs from the ego's
// ((d0, d1) != 0; every agent hit has s > 0): gamma (H - dmin) [+ L_f], so that row_b =
// row_g + c.  Bit for bit row_b's H: with s = sign(d), s d0 = |d0| up to the sign of a zero, and
// a zero's sign cannot reach |d0| + |d1| once either is nonzero; k s is k or -k exactly.  The
// per-quadrant minimum can then be taken over row_g and c added once per quadrant: x -> x + c
// rounds monotonically, so min_j (g_j + c) = (min_j g_j) + c exactly whenever c is finite (the
// caller checks that; a NaN g_j is skipped by both minima).
template <bool FZ = false>
__device__ __forceinline__ double row_g(const KP& P, const Ego& E, double o0, double o1, double o2, double o3,
                                        int& q) {
    const double d0 = E.r0 - o0, d1 = E.r1 - o1, d2 = E.r2 - o2, d3 = E.r3 - o3;
    const bool nx = d0 < 0, ny = d1 < 0;
    const double ksx = nx ? -P.k : P.k, ksy = ny ? -P.k : P.k;
    const double H = fma(ksy, d3, fma(ksx, d2, fabs(d0) + fabs(d1)));
    q = (nx ? 1 : 0) | (ny ? 2 : 0);
    if (FZ) return P.gamma * (H - P.dmin);
    double Lf = 0.0;
    if (!P.f_zero) Lf = lf_term(P, d0, d1, d2, d3, nx ? -1.0 : 1.0, ny ? -1.0 : 1.0, ksx, ksy);
    return P.gamma * (H - P.dmin) + Lf;
}

template <bool FZ = false>
__device__ __forceinline__ void ego_add(const KP& P, Ego& E, double o0, double o1, double o2, double o3) {
    int q;
    const double b = row_b<FZ>(P, E, o0, o1, o2, o3, q);
    // four predicated compare-selects: keeps bq0..3 in registers (a select-then-write-back form
    // gets lowered to a dynamically indexed private array, i.e. scratch)
    E.bq0 = (q == 0 && b < E.bq0) ? b : E.bq0;
    E.bq1 = (q == 1 && b < E.bq1) ? b : E.bq1;
    E.bq2 = (q == 2 && b < E.bq2) ? b : E.bq2;
    E.bq3 = (q == 3 && b < E.bq3) ? b : E.bq3;
    E.present |= 1u << q;
    E.count++;
}

// Per-lane list of cull hits in LDS (column per lane: conflict-free), flushed into the ego's QP
// after the scan.  More than kHitCap hits -> the caller rescans with direct assembly.
#ifndef CBF_HIT_CAP
#define CBF_HIT_CAP 16
#endif
// Slot t of a cell-sorted array through a 32-bit byte offset from the (uniform) base: one address
// instruction per load instead of a 64-bit multiply-add.  The lattice entry points bound windows
// to < 2^28 slots (check_lattice), so 16 t fits in 32 bits.
__device__ __forceinline__ double2 ld_slot(const double2* __restrict__ a, int t) {
    return *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(a) + ((uint32_t)t << 4));
}
constexpr int kHitCap = CBF_HIT_CAP;
struct HitList {
    int n = 0;
    __device__ __forceinline__ void push(int* lds, int t) {
        if (n < kHitCap) lds[n * kBlock + threadIdx.x] = t;
        ++n;
    }
    __device__ __forceinline__ bool overflowed() const { return n > kHitCap; }
    // flush into the per-quadrant minima of row_g kept in LDS (gq[q * kBlock + lane], preset to
    // +inf by the caller, which adds the quadrant terms c after): one read-compare-write per hit
    // instead of four register compare-selects; same rows, same minimum (row_g).  Agent hits only
    // (s > 0).
    template <bool FZ = false>
    __device__ __forceinline__ void flush_gq(const int* lds, double* gq, const KP& P, Ego& E,
                                             const double2* __restrict__ pos, const double2* __restrict__ vel) {
        for (int i = 0; i < n; i += CBF_FLUSH_U) {
            double2 pj[CBF_FLUSH_U], vj[CBF_FLUSH_U];
#pragma unroll
            for (int q = 0; q < CBF_FLUSH_U; ++q) {
                if (i + q < n) {
                    const int t = lds[(i + q) * kBlock + threadIdx.x];
                    pj[q] = ld_slot(pos, t);
                    vj[q] = ld_slot(vel, t);
                }
            }
#pragma unroll
            for (int q = 0; q < CBF_FLUSH_U; ++q) {
                if (i + q < n) {
                    int qd;
                    const double g = row_g<FZ>(P, E, pj[q].x, pj[q].y, vj[q].x, vj[q].y, qd);
                    double* slot = gq + qd * kBlock + threadIdx.x;
                    *slot = vmin_f64(*slot, g);  // = (g < cur ? g : cur): see vmin_f64
                    E.present |= 1u << qd;
                }
            }
        }
        E.count += n;
        n = 0;
    }
};

// The three cell-row ranges of an ego scanned as one sequence, CBF_SCAN_U candidates' loads in
// flight per lane; hits (0 < s < cull_t, cross_and_rescue.py:147-150) go to the hit list in
// sequence order.  smin tracks the smallest hit distance^2 (the rollout's minimum pairwise
// distance, a reported statistic only).
__device__ __forceinline__ void scan_rows_joint(const int (&t0)[3], const int (&t1)[3], const KP& P, const Ego& E,
                                                HitList& H, int* lds, const double2* __restrict__ spos,
                                                double& smin) {
    const int l0 = t1[0] - t0[0], l01 = l0 + (t1[1] - t0[1]);
    const int L = l01 + (t1[2] - t0[2]);
    for (int v = 0; v < L; v += CBF_SCAN_U) {
        double2 p[CBF_SCAN_U];
        int tt[CBF_SCAN_U];
#pragma unroll
        for (int q = 0; q < CBF_SCAN_U; ++q) {
            const int vv = v + q;
            tt[q] = vv < l0 ? t0[0] + vv : (vv < l01 ? t0[1] + (vv - l0) : t0[2] + (vv - l01));
            if (vv < L) p[q] = ld_slot(spos, tt[q]);
        }
#pragma unroll
        for (int q = 0; q < CBF_SCAN_U; ++q) {
            if (v + q < L) {
                const double e0 = p[q].x - E.r0, e1 = p[q].y - E.r1;
                const double s = e0 * e0 + e1 * e1;
                if (s < P.cull_t && s > 0) {
                    H.push(lds, tt[q]);
                    smin = pmin(smin, s);
                }
            }
        }
    }
}

// Direct (uncompacted) cull + assembly over [t0, t1): the overflow path.
template <bool FZ = false>
__device__ __forceinline__ void scan_range_direct(int t0, int t1, const KP& P, Ego& E,
                                                  const double2* __restrict__ spos,
                                                  const double2* __restrict__ svel) {
    for (int t = t0; t < t1; ++t) {
        const double2 pj = spos[t];
        const double e0 = pj.x - E.r0, e1 = pj.y - E.r1;
        const double s = e0 * e0 + e1 * e1;
        if (!(s < P.cull_t && s > 0)) continue;
        const double2 vj = svel[t];
        ego_add<FZ>(P, E, pj.x, pj.y, vj.x, vj.y);
    }
}

// Cull test (cross_and_rescue.py:141-150): sqrt(s) < d <=> s < cull_t; agents also need s > 0.
__device__ __forceinline__ bool cull_keep(const KP& P, double r0, double r1, double p0, double p1, bool is_obstacle,
                                          double& s) {
    const double e0 = p0 - r0, e1 = p1 - r1;
    s = e0 * e0 + e1 * e1;
    return s < P.cull_t && (is_obstacle || s > 0);
}

// Box rows S_saturated (cbf.py:67-70), reference row order.
struct Box {
    double S[8];
};
__device__ __forceinline__ Box box_rhs(const KP& P, const Ego& E) {
    Box B;
    const double ms = P.ms;
    B.S[0] = ms - E.u0x;
    B.S[1] = ms + E.u0x;
    B.S[2] = ms - E.u0y;
    B.S[3] = ms + E.u0y;
    B.S[4] = (ms - E.r2) - E.u0x;
    B.S[5] = (ms + E.r2) + E.u0x;
    B.S[6] = (ms - E.r3) - E.u0y;
    B.S[7] = (ms + E.r3) + E.u0y;
    return B;
}

// Exact min-norm point of the (<= N) half-planes a.x <= b whose slot bit is set in mask, in slot
// order; slots 0..3 are the merged box rows.  Incremental (Seidel) method, identical arithmetic
// to oracle/cbf_oracle.c:solve_planes_n over the present planes.  All loops are unrolled over
// the N slots so the planes stay in registers.  Returns -1 (feasible) or the slot at which the
// prefix became infeasible.
template <int N>
__device__ __forceinline__ int solve_planes_reg(const double (&a0)[N], const double (&a1)[N], const double (&b)[N],
                                                unsigned mask, double& xo0, double& xo1) {
    double tb[N];
#pragma unroll
    for (int h = 0; h < N; ++h) tb[h] = FEAS_TOL * max1abs(b[h]);
    double x0 = 0.0, x1 = 0.0;
#pragma unroll
    for (int h = 0; h < N; ++h) {
        if (!((mask >> h) & 1u)) continue;
        if ((a0[h] * x0 + a1[h] * x1) - b[h] <= tb[h]) continue;
        const double n2 = a0[h] * a0[h] + a1[h] * a1[h];
        if (!(n2 > 0)) return h;
        const double t = b[h] / n2;
        const double p0 = t * a0[h], p1 = t * a1[h];
        const double d0 = -a1[h], d1 = a0[h];
        // 1-D interval on the line: upper bounds r/ad (ad > 0), lower bounds r/ad (ad < 0),
        // compared by cross-multiplication; only the binding bound is divided out.
        double rh = 0.0, ah = 0.0, rl = 0.0, al = 0.0;
        bool has_hi = false, has_lo = false;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            if (!((mask >> j) & 1u)) continue;
            const double ad = a0[j] * d0 + a1[j] * d1;
            const double r = b[j] - (a0[j] * p0 + a1[j] * p1);
            if (ad > 0) {
                if (!has_hi || r * ah < rh * ad) {
                    rh = r;
                    ah = ad;
                }
                has_hi = true;
            } else if (ad < 0) {
                if (!has_lo || r * al > rl * ad) {
                    rl = r;
                    al = ad;
                }
                has_lo = true;
            }
        }
        double s = 0.0;
        bool s_hi = false;
        if (has_hi && rh < 0) {  // hi = rh/ah < 0
            s = rh / ah;
            s_hi = true;
        }
        if (has_lo && (s_hi ? (rh * al > rl * ah) : (rl < 0)))  // s < lo = rl/al
            s = rl / al;
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j <= h; ++j)
            if ((mask >> j) & 1u) ok = ok && ((a0[j] * x0 + a1[j] * x1) - b[j] <= tb[j]);
        if (!ok) return h;
    }
    xo0 = x0;
    xo1 = x1;
    return -1;
}

// slots 0..3: merged box rows, 4..7: the CBF quadrants
__device__ __forceinline__ int solve8(const double (&a0)[8], const double (&a1)[8], const double (&b)[8],
                                      unsigned mask, double& xo0, double& xo1) {
    return solve_planes_reg<8>(a0, a1, b, mask, xo0, xo1);
}

struct Sol {
    double x0, x1;
    int status;
    int iters;
    double viol;       // max(0, a.x - b) over the rows of the QP actually solved (relaxed rhs)
    double viol_orig;  // the same over the ORIGINAL rows (cbf.py:58-59 before any +1, box rows)
};

// max(0, max_i a_i.x - b_i) over an ego's original rows: the merged box rows and the per-quadrant
// barrier minima before relaxation.  Equal to Sol::viol for an OPTIMAL QP; for a RELAXED one it is
// how far the returned control violates the barrier the reference asked for (a reported
// statistic).
__device__ __forceinline__ double orig_violation(const KP& P, const Ego& E, const Box& B, double x0, double x1) {
    double v = 0.0;
    const double bb[4] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7])};
    const double ab[4] = {x0, x1, -x0, -x1};
#pragma unroll
    for (int h = 0; h < 4; ++h) v = pmax(v, ab[h] - bb[h]);
    const double bq[4] = {E.bq0, E.bq1, E.bq2, E.bq3};
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if ((E.present >> q) & 1u) v = pmax(v, (P.n0[q] * x0 + P.n1[q] * x1) - bq[q]);
    return v;
}

// The QP of cbf.py:62-87 for an ego: merged box rows + per-quadrant CBF rows, with the
// reference's +1 relaxation (cbf.py:84-87) applied while infeasible.
__device__ __forceinline__ Sol solve_ego(const KP& P, const Ego& E) {
    const Box B = box_rhs(P, E);
    double a0[8] = {1.0, 0.0, -1.0, 0.0, P.n0[0], P.n0[1], P.n0[2], P.n0[3]};
    double a1[8] = {0.0, 1.0, 0.0, -1.0, P.n1[0], P.n1[1], P.n1[2], P.n1[3]};
    double b[8] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7]),
                   E.bq0, E.bq1, E.bq2, E.bq3};
    const unsigned mask = 0xFu | (E.present << 4);
    Sol S;
    S.status = CBF_STATUS_OPTIMAL;
    S.iters = 0;
    S.x0 = S.x1 = 0.0;
    // Strip pre-check: quadrants q and 3-q have exactly opposite normals (negation is exact in
    // IEEE), so both rows can hold within tolerance only if b_q + b_{3-q} >= -(tb_q + tb_{3-q}).
    // While that is violated by a clear margin the exact solve below is certain to fail at a CBF
    // plane, so skip it and apply the +1 relaxation directly -- same iterates, same result as
    // solving at every count (the oracle does; tests check bit-equality).
    if ((E.present & 9u) == 9u || (E.present & 6u) == 6u) {
        for (;;) {
            bool dead = false;
            if ((E.present & 9u) == 9u) {
                const double s = b[4] + b[7];
                const double tb = FEAS_TOL * (max1abs(b[4]) + max1abs(b[7]));
                dead = dead || (s < -tb - 1e-9 * (1.0 + fabs(b[4]) + fabs(b[7])));
            }
            if ((E.present & 6u) == 6u) {
                const double s = b[5] + b[6];
                const double tb = FEAS_TOL * (max1abs(b[5]) + max1abs(b[6]));
                dead = dead || (s < -tb - 1e-9 * (1.0 + fabs(b[5]) + fabs(b[6])));
            }
            if (!dead || S.iters >= P.relax_cap) break;
            b[4] = b[4] + 1.0;
            b[5] = b[5] + 1.0;
            b[6] = b[6] + 1.0;
            b[7] = b[7] + 1.0;
            S.iters++;
        }
    }
    for (;;) {
        const int fail = solve8(a0, a1, b, mask, S.x0, S.x1);
        if (fail < 0) break;
        if (fail < 4) {  // reported as at the first solve: no relaxation applied
            S.status = CBF_STATUS_BOX_INFEASIBLE;
            S.iters = 0;
            S.x0 = S.x1 = 0.0;
            b[4] = E.bq0;
            b[5] = E.bq1;
            b[6] = E.bq2;
            b[7] = E.bq3;
            break;
        }
        if (S.iters >= P.relax_cap) {
            S.status = CBF_STATUS_RELAX_CAP;
            S.x0 = S.x1 = 0.0;
            break;
        }
        b[4] = b[4] + 1.0;
        b[5] = b[5] + 1.0;
        b[6] = b[6] + 1.0;
        b[7] = b[7] + 1.0;
        S.iters++;
    }
    if (S.status == CBF_STATUS_OPTIMAL && S.iters > 0) S.status = CBF_STATUS_RELAXED;
    double v = 0.0;
#pragma unroll
    for (int h = 0; h < 8; ++h)
        if ((mask >> h) & 1u) {
            const double d = (a0[h] * S.x0 + a1[h] * S.x1) - b[h];
            if (d > v) v = d;
        }
    S.viol = v;
    S.viol_orig = S.iters > 0 ? orig_violation(P, E, B, S.x0, S.x1) : v;
    return S;
}

// The common cases of solve_ego without the full Seidel machinery, bit-identical to it.  After the
// strip pre-relaxation, solve_ego's first solve8 call either finds the origin feasible (no plane
// violated: x = 0), or meets exactly one violated plane h whose projection p = (b_h / |a_h|^2) a_h
// is not moved along the line (every earlier plane j with a_j.d != 0 has b_j - a_j.p >= 0, so the
// 1-D bound search keeps s = 0) and satisfies every plane within tolerance, so that solve8 returns
// x = p + 0 d there.  Both are decided with solve8's own expressions; anything else (a second
// event, a bound that moves x, an infeasible prefix, non-finite data) returns false and the caller
// runs solve_ego.  Measured: 57 % (cfg4) and 89 % (cfg4f) of the QPs the origin does not solve are
// one such event (tools).
// solve_fast in two stages: the strip pre-relaxation and solve8's test at the origin
// (fast_origin: returns true with S set when the origin is the answer), then the one-event check
// (fast_event).  The filter kernels that defer the second stage to a few lanes (the window tile's
// event queue) call them apart.
struct FastState {
    Box B;
    double b[8];
    int iters, h;
    double v0;
};
__device__ __forceinline__ bool fast_origin(const KP& P, const Ego& E, FastState& F, Sol& S) {
    F.B = box_rhs(P, E);
    const Box& B = F.B;
    const double a0[8] = {1.0, 0.0, -1.0, 0.0, P.n0[0], P.n0[1], P.n0[2], P.n0[3]};
    const double a1[8] = {0.0, 1.0, 0.0, -1.0, P.n1[0], P.n1[1], P.n1[2], P.n1[3]};
    double* b = F.b;
    b[0] = pmin(B.S[0], B.S[4]);
    b[1] = pmin(B.S[1], B.S[6]);
    b[2] = pmin(B.S[2], B.S[5]);
    b[3] = pmin(B.S[3], B.S[7]);
    b[4] = E.bq0;
    b[5] = E.bq1;
    b[6] = E.bq2;
    b[7] = E.bq3;
    const unsigned mask = 0xFu | (E.present << 4);
    int iters = 0;
    if ((E.present & 9u) == 9u || (E.present & 6u) == 6u) {  // strip pre-check, as solve_ego
        for (;;) {
            bool dead = false;
            if ((E.present & 9u) == 9u) {
                const double s = b[4] + b[7];
                const double tb = FEAS_TOL * (max1abs(b[4]) + max1abs(b[7]));
                dead = dead || (s < -tb - 1e-9 * (1.0 + fabs(b[4]) + fabs(b[7])));
            }
            if ((E.present & 6u) == 6u) {
                const double s = b[5] + b[6];
                const double tb = FEAS_TOL * (max1abs(b[5]) + max1abs(b[6]));
                dead = dead || (s < -tb - 1e-9 * (1.0 + fabs(b[5]) + fabs(b[6])));
            }
            if (!dead || iters >= P.relax_cap) break;
            b[4] = b[4] + 1.0;
            b[5] = b[5] + 1.0;
            b[6] = b[6] + 1.0;
            b[7] = b[7] + 1.0;
            iters++;
        }
    }
    // the first plane violated at the origin (solve8's test at x = 0), and the origin's violation
    int h = -1;
    double v0 = 0.0;
#pragma unroll
    for (int j = 7; j >= 0; --j)
        if ((mask >> j) & 1u) {
            // a.0 for the CBF planes from the host (P.z: the same products and sum, uniform)
            const double d = (j < 4 ? (a0[j] * 0.0 + a1[j] * 0.0) : P.z[j - 4]) - b[j];
            if (!(d <= FEAS_TOL * max1abs(b[j]))) h = j;
            if (d > v0) v0 = d;
        }
    F.iters = iters;
    F.h = h;
    F.v0 = v0;
    if (h < 0) {  // solve8 returns the origin; the final check below would repeat the test above
        S.x0 = 0.0;
        S.x1 = 0.0;
        S.iters = iters;
        S.status = iters > 0 ? CBF_STATUS_RELAXED : CBF_STATUS_OPTIMAL;
        S.viol = v0;
        S.viol_orig = iters > 0 ? orig_violation(P, E, B, 0.0, 0.0) : v0;
        return true;
    }
    return false;
}
__device__ __forceinline__ bool fast_event(const KP& P, const Ego& E, const FastState& F, Sol& S) {
    const double a0[8] = {1.0, 0.0, -1.0, 0.0, P.n0[0], P.n0[1], P.n0[2], P.n0[3]};
    const double a1[8] = {0.0, 1.0, 0.0, -1.0, P.n1[0], P.n1[1], P.n1[2], P.n1[3]};
    const double* b = F.b;
    const unsigned mask = 0xFu | (E.present << 4);
    const int h = F.h;
    double x0 = 0.0, x1 = 0.0;
    {
        double ah0 = 0.0, ah1 = 0.0, bh = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j == h) {
                ah0 = a0[j];
                ah1 = a1[j];
                bh = b[j];
            }
        const double n2 = ah0 * ah0 + ah1 * ah1;
        if (!(n2 > 0)) return false;
        const double t = bh / n2;
        const double p0 = t * ah0, p1 = t * ah1;
        const double d0 = -ah1, d1 = ah0;
        bool stay = true;  // the 1-D bound search over planes j < h keeps s = 0
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j >= h || !((mask >> j) & 1u)) continue;
            const double ad = a0[j] * d0 + a1[j] * d1;
            const double r = b[j] - (a0[j] * p0 + a1[j] * p1);
            if ((ad > 0 || ad < 0) && !(r >= 0)) stay = false;
        }
        if (!stay) return false;
        const double s0 = 0.0;
        x0 = p0 + s0 * d0;
        x1 = p1 + s0 * d1;
    }
    bool ok = true;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((mask >> j) & 1u) {
            const double d = (a0[j] * x0 + a1[j] * x1) - b[j];
            ok = ok && (d <= FEAS_TOL * max1abs(b[j]));
            if (d > v) v = d;
        }
    if (!ok) return false;
    S.x0 = x0;
    S.x1 = x1;
    S.iters = F.iters;
    S.status = F.iters > 0 ? CBF_STATUS_RELAXED : CBF_STATUS_OPTIMAL;
    S.viol = v;
    S.viol_orig = F.iters > 0 ? orig_violation(P, E, F.B, x0, x1) : v;
    return true;
}
__device__ __forceinline__ bool solve_fast(const KP& P, const Ego& E, Sol& S) {
    FastState F;
    if (fast_origin(P, E, F, S)) return true;
    return fast_event(P, E, F, S);
}

// cbf.py:89-91
__device__ __forceinline__ void clip_u(const KP& P, const Sol& S, const Ego& E, double& ux, double& uy) {
    ux = pmax(pmin(S.x0 + E.u0x, P.ms), -P.ms);
    uy = pmax(pmin(S.x1 + E.u0y, P.ms), -P.ms);
}

__device__ __forceinline__ int32_t pack_status(const Sol& S) {
    const int it = S.iters < (1 << 23) ? S.iters : (1 << 23) - 1;
    return S.status | (it << 8);
}

// Active-row test at x for a neighbour row after `iters` relaxations (SURVEY 8d gate).
__device__ __forceinline__ uint8_t row_active(const KP& P, const Ego& E, const Sol& S, double o0, double o1,
                                              double o2, double o3) {
    int q;
    double b = row_b(P, E, o0, o1, o2, o3, q);
    for (int i = 0; i < S.iters; ++i) b = b + 1.0;
    double a0 = 0, a1 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (q == k) {
            a0 = P.n0[k];
            a1 = P.n1[k];
        }
    const double lhs = a0 * S.x0 + a1 * S.x1;
    return lhs >= b - ACTIVE_TOL * pmax(1.0, fabs(b)) ? 1 : 0;
}

__device__ __forceinline__ uint8_t box_active_bits(const KP& P, const Ego& E, const Sol& S) {
    const Box B = box_rhs(P, E);
    const double g0[8] = {1.0, 0.0, -1.0, 0.0, 1.0, -1.0, 0.0, 0.0};
    const double g1[8] = {0.0, 1.0, 0.0, -1.0, 0.0, 0.0, 1.0, -1.0};
    uint8_t bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double lhs = g0[i] * S.x0 + g1[i] * S.x1;
        if (lhs >= B.S[i] - ACTIVE_TOL * pmax(1.0, fabs(B.S[i]))) bits |= (uint8_t)(1u << i);
    }
    return bits;
}

// Uniform-grid cell coordinate with clamping (exact for any input; NaN -> 0).
__device__ __forceinline__ int cell_coord(double v, double o, double inv_h, int n) {
    double f = floor((v - o) * inv_h);
    if (!(f >= 0.0)) f = 0.0;
    if (f > (double)(n - 1)) f = (double)(n - 1);
    return (int)f;
}

// Monotone u64 key of a double (for atomicMin/Max extents).
__device__ __forceinline__ unsigned long long dkey(double v) {
    unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

}  // namespace cbf
