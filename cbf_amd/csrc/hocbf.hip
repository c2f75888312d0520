// hocbf.hip -- Euclidean HOCBF barrier mode on gfx950 (BASELINE.json north star (2); SURVEY 8f
// rank 4).  The reference's barrier is the sign-switched L1 form of cbf.py:38-59; this mode swaps
// it for h_ij = |p_i - p_j|^2 - Ds^2 with its relative-degree-2 psi terms (double integrator
// p' = v, v' = u, neighbours at constant velocity):
//     (-2 dp) . u  <=  2|dv|^2 + (a1 + a2) h' + a1 a2 h,   h' = 2 dp.dv,
// keeping everything else of get_safe_control (box rows, +1 relaxation, de-bias, clip).  Every
// barrier row is its own half-plane, so the exact 2-D solve is the general incremental one over
// 4 box planes + m rows (rows live in a caller workspace, 32 B each, relaxed in place).  Same
// arithmetic, order and tolerances as oracle/cbf_oracle.c (hocbf_row / solve_hocbf), so results
// are bit-identical to the oracle.
#include "cbf_device.hpp"
#include "cells.hpp"
#include "lattice.hpp"

using namespace cbf;

extern "C" __device__ __attribute__((const)) double __ockl_wfred_min_f64(double);

namespace {

struct HP {
    double a_sum, a_prod;  // alpha1 + alpha2, alpha1 * alpha2 (fp64, as the oracle forms them)
};

__device__ __forceinline__ double4 hocbf_row(const KP& P, const HP& H, double r0, double r1, double r2, double r3,
                                             double o0, double o1, double o2, double o3, double u0x, double u0y) {
    const double dx = r0 - o0, dy = r1 - o1, dvx = r2 - o2, dvy = r3 - o3;
    const double h = (dx * dx + dy * dy) - P.dmin * P.dmin;
    const double hd = 2.0 * (dx * dvx + dy * dvy);
    const double vv = dvx * dvx + dvy * dvy;
    const double rhs = (2.0 * vv + H.a_sum * hd) + H.a_prod * h;
    const double a0 = -2.0 * dx, a1 = -2.0 * dy;
    return make_double4(a0, a1, rhs - (a0 * u0x + a1 * u0y), 0.0);
}


#ifndef CBF_HOCBF_CERT
#define CBF_HOCBF_CERT 1  // 0: every relaxation pass run in the main kernel, no infeasibility certificate
#endif
#ifndef CBF_HOCBF_HARD_BATCHED
#define CBF_HOCBF_HARD_BATCHED 1  // the hard role's solve with batched row loads (0: solve_hocbf's loops)
#endif
#ifndef CBF_HOCBF_CERT_J
#define CBF_HOCBF_CERT_J 1  // partners j tried with every third row (2: the best two; main kernel
                            // 80.9 against 73.3 us at cfg4, the hard role 42.3 against 43.1)
#endif
#ifndef CBF_HOCBF_UNROLL
#define CBF_HOCBF_UNROLL 8  // solve_rows' inner loops over the earlier rows, unrolled
#endif

// Plane source over rows stored in memory (workspace), relaxed in place.
struct StoredRows {
    double4* rows;
    int m;
    __device__ __forceinline__ void row(int i, double& a0, double& a1, double& b) const {
        const double4 r = rows[i];
        a0 = r.x;
        a1 = r.y;
        b = r.z;
    }
    __device__ __forceinline__ void relax() {
        for (int i = 0; i < m; ++i) rows[i].z = rows[i].z + 1.0;  // cbf.py:85-87
    }
};

// Plane source recomputing each row from the neighbour's cell-sorted state (lattice step); the
// neighbours are LDS keys (entity << 32 | slot) in ascending entity order; `t` relaxations are
// re-applied as t successive +1 additions (the oracle's rounding sequence).
struct SlotRows {
    const KP& P;
    const HP& H;
    const Ego& E;
    const unsigned long long* keys;  // keys[i * ks + lane]
    int ks, lane;
    const double2* __restrict__ spos;
    const double2* __restrict__ svel;
    int m;
    int t;
    __device__ __forceinline__ void row(int i, double& a0, double& a1, double& b) const {
        const int slot = (int)(keys[i * ks + lane] & 0xFFFFFFFFull);
        const double2 o = spos[slot], ov = svel[slot];
        const double4 r = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, o.x, o.y, ov.x, ov.y, E.u0x, E.u0y);
        a0 = r.x;
        a1 = r.y;
        b = r.z;
        for (int k = 0; k < t; ++k) b = b + 1.0;
    }
    __device__ __forceinline__ void relax() { ++t; }
};

__device__ __forceinline__ bool feas(double a0, double a1, double b, double x0, double x1) {
    return (a0 * x0 + a1 * x1) - b <= FEAS_TOL * pmax(1.0, fabs(b));
}

// 1-D interval of the incremental solve: bounds r/ad compared by cross-multiplication, only the
// binding one divided out (oracle/cbf_oracle.c:solve_planes_n, inner loop).
struct Interval {
    double rh = 0.0, ah = 0.0, rl = 0.0, al = 0.0;
    bool has_hi = false, has_lo = false;
    __device__ __forceinline__ void add(double c0, double c1, double e, double d0, double d1, double p0, double p1) {
        const double ad = c0 * d0 + c1 * d1;
        const double r = e - (c0 * p0 + c1 * p1);
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
    __device__ __forceinline__ double clamp0() const {
        double s = 0.0;
        bool s_hi = false;
        if (has_hi && rh < 0) {
            s = rh / ah;
            s_hi = true;
        }
        if (has_lo && (s_hi ? (rh * al > rl * ah) : (rl < 0))) s = rl / al;
        return s;
    }
};

// oracle/cbf_oracle.c:solve_planes_n over the 4 merged box planes (static, in registers) then the
// m barrier rows of R (dynamic), in that order; same arithmetic.  The box planes are never
// selected by a runtime index (that would be lowered to scratch).
// The box planes' part of solve_rows (h = 0..3, from x = 0): the failing plane, or -1 with x set.
// It depends on the box alone, so it is the same in every pass of the relaxation loop.
__device__ __forceinline__ int box_phase(const double (&bb)[4], double& x0, double& x1) {
    const double ba0[4] = {1.0, 0.0, -1.0, 0.0}, ba1[4] = {0.0, 1.0, 0.0, -1.0};
    x0 = 0.0;
    x1 = 0.0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        if (feas(ba0[h], ba1[h], bb[h], x0, x1)) continue;
        const double n2 = ba0[h] * ba0[h] + ba1[h] * ba1[h];
        const double t = bb[h] / n2;
        const double p0 = t * ba0[h], p1 = t * ba1[h];
        const double d0 = -ba1[h], d1 = ba0[h];
        Interval I;
#pragma unroll
        for (int j = 0; j < h; ++j) I.add(ba0[j], ba1[j], bb[j], d0, d1, p0, p1);
        const double s = I.clamp0();
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j <= h; ++j) ok = ok && feas(ba0[j], ba1[j], bb[j], x0, x1);
        if (!ok) return h;
    }
    return -1;
}

template <class Src>
__device__ __forceinline__ int solve_rows(const double (&bb)[4], const Src& R, double& xo0, double& xo1) {
    const double ba0[4] = {1.0, 0.0, -1.0, 0.0}, ba1[4] = {0.0, 1.0, 0.0, -1.0};
    double x0, x1;
    // box planes h = 0..3
    const int hb = box_phase(bb, x0, x1);
    if (hb >= 0) return hb;
    // barrier rows h = 4 + i
    for (int i = 0; i < R.m; ++i) {
        double a0, a1, b;
        R.row(i, a0, a1, b);
        if (feas(a0, a1, b, x0, x1)) continue;
        const double n2 = a0 * a0 + a1 * a1;
        if (!(n2 > 0)) return 4 + i;
        const double t = b / n2;
        const double p0 = t * a0, p1 = t * a1;
        const double d0 = -a1, d1 = a0;
        Interval I;
#pragma unroll
        for (int j = 0; j < 4; ++j) I.add(ba0[j], ba1[j], bb[j], d0, d1, p0, p1);
#pragma unroll CBF_HOCBF_UNROLL
        for (int j = 0; j < i; ++j) {  // (unrolled: the rows' LDS loads issue together)
            double c0, c1, e;
            R.row(j, c0, c1, e);
            I.add(c0, c1, e, d0, d1, p0, p1);
        }
        const double s = I.clamp0();
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok = ok && feas(ba0[j], ba1[j], bb[j], x0, x1);
        if (!ok) return 4 + i;
#pragma unroll CBF_HOCBF_UNROLL
        for (int j = 0; j <= i; ++j) {
            double c0, c1, e;
            R.row(j, c0, c1, e);
            if (!feas(c0, c1, e, x0, x1)) return 4 + i;
        }
    }
    xo0 = x0;
    xo1 = x1;
    return -1;
}

// Infeasibility certificate for the unrelaxed rows (Farkas, three rows): if it holds, the first
// pass of solve_hocbf is certain to fail at a barrier row, so the caller may start at one
// relaxation -- the same state the failed pass leaves (iters 1, RELAXED; box phase checked apart).
// Proof: a pass that succeeds ends at an x meeting every plane within feas' tolerance, i.e. (real
// arithmetic) a_t.x - b_t <= tau_t with tau_t <= 1.01e-12 max(1, |b_t|) + 4u (|a_t0||x0| +
// |a_t1||x1| + |b_t|), and the box planes likewise, so |x0| <= X0, |x1| <= X1 below.  For any
// lambda >= 0 summing the rows gives R.x - sum lambda b <= sum lambda tau with R = sum lambda a, and
// R.x >= -(|R0| X0 + |R1| X1); so sum lambda b + |R0| X0 + |R1| X1 + sum lambda tau < 0 rules every
// such x out.  The test below asks that sum, evaluated in fp64, to be below -1e-9 mag (mag = sum
// lambda (1 + |b| + |a0| X0 + |a1| X1)), which bounds every tau and every rounding error of the
// evaluation (each <= 1e-11 mag) with room to spare.  lambda: the cross products of the three rows
// (sum lambda a = 0 in real arithmetic; used only when all share a sign).  Non-finite data never
// passes (a NaN or inf comparison is false).
struct CertRow {
    double a0, a1, b, mg;  // the row and its share of mag per unit lambda
};
__device__ __forceinline__ bool cert_triple(const CertRow& I, const CertRow& J, const CertRow& K, double X0,
                                            double X1) {
    double li = J.a0 * K.a1 - J.a1 * K.a0, lj = K.a0 * I.a1 - K.a1 * I.a0, lk = I.a0 * J.a1 - I.a1 * J.a0;
    const bool pos = li >= 0.0 && lj >= 0.0 && lk >= 0.0, neg = li <= 0.0 && lj <= 0.0 && lk <= 0.0;
    if (neg) {
        li = -li;
        lj = -lj;
        lk = -lk;
    }
    const double sb = (li * I.b + lj * J.b) + lk * K.b;
    const double r0 = (li * I.a0 + lj * J.a0) + lk * K.a0, r1 = (li * I.a1 + lj * J.a1) + lk * K.a1;
    const double mag = (li * I.mg + lj * J.mg) + lk * K.mg;
    const double q = (sb + fabs(r0) * X0) + fabs(r1) * X1;
    return (pos || neg) && q < -1e-9 * mag;
}
__device__ __forceinline__ CertRow cert_row(double a0, double a1, double b, double X0, double X1) {
    return CertRow{a0, a1, b, 1.0 + fabs(b) + fabs(a0) * X0 + fabs(a1) * X1};
}
__device__ __forceinline__ void cert_bounds(const double (&bb)[4], double& X0, double& X1) {
    X0 = pmax(fabs(bb[0]), fabs(bb[2])) * (1.0 + 1e-11) + 1e-11;
    X1 = pmax(fabs(bb[1]), fabs(bb[3])) * (1.0 + 1e-11) + 1e-11;
}

// oracle/cbf_oracle.c:solve_hocbf -- +1 relaxation of every barrier row while infeasible
template <class Src>
__device__ __forceinline__ Sol solve_hocbf(const KP& P, const Ego& E, Src& R) {
    const Box B = box_rhs(P, E);
    const double bb[4] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7])};
    Sol S;
    S.status = CBF_STATUS_OPTIMAL;
    S.iters = 0;
    S.x0 = S.x1 = 0.0;
    S.viol = 0.0;
    for (;;) {
        const int fail = solve_rows(bb, R, S.x0, S.x1);
        if (fail < 0) break;
        if (fail < 4) {
            S.status = CBF_STATUS_BOX_INFEASIBLE;
            S.x0 = S.x1 = 0.0;
            break;
        }
        if (S.iters >= P.relax_cap) {
            S.status = CBF_STATUS_RELAX_CAP;
            S.x0 = S.x1 = 0.0;
            break;
        }
        R.relax();
        S.iters++;
        S.status = CBF_STATUS_RELAXED;
    }
    return S;
}

// Plane source over rows staged per lane in LDS (the lattice kernel's key area, reused once the
// keys are in registers): row i's a0, a1, b at lds[(3i + c) * ks + lane]; relaxed in place.
constexpr int kLdsRows = 8;
struct LdsRows {
    double* lds;
    int ks, lane;
    int m;
    __device__ __forceinline__ void row(int i, double& a0, double& a1, double& b) const {
        a0 = lds[(3 * i) * ks + lane];
        a1 = lds[(3 * i + 1) * ks + lane];
        b = lds[(3 * i + 2) * ks + lane];
    }
    __device__ __forceinline__ void relax() {
#pragma unroll CBF_HOCBF_UNROLL
        for (int i = 0; i < m; ++i) {
            double& v = lds[(3 * i + 2) * ks + lane];
            v = v + 1.0;  // cbf.py:85-87
        }
    }
};

// get_safe_control with explicit neighbour lists (CSR): rows of ego i at ws[off[i] .. off[i+1])
__global__ void __launch_bounds__(kBlock) k_hocbf_batch(KP P, HP H, int n, const double* __restrict__ rs,
                                                        const double* __restrict__ u0, const int32_t* __restrict__ off,
                                                        const double* __restrict__ obs, double* __restrict__ u,
                                                        int32_t* __restrict__ status, double* __restrict__ xo,
                                                        double4* __restrict__ ws) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double2 ra = reinterpret_cast<const double2*>(rs)[2 * i];
    const double2 rb = reinterpret_cast<const double2*>(rs)[2 * i + 1];
    const double2 uu = reinterpret_cast<const double2*>(u0)[i];
    Ego E;
    ego_init(P, E, ra.x, ra.y, rb.x, rb.y, uu.x, uu.y);
    const int t0 = off[i], m = off[i + 1] - off[i];
    double4* rows = ws + t0;
    for (int t = 0; t < m; ++t) {
        const double2 oa = reinterpret_cast<const double2*>(obs)[2 * (t0 + t)];
        const double2 ob = reinterpret_cast<const double2*>(obs)[2 * (t0 + t) + 1];
        rows[t] = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, oa.x, oa.y, ob.x, ob.y, E.u0x, E.u0y);
    }
    StoredRows R{rows, m};
    const Sol S = solve_hocbf(P, E, R);
    double ux, uy;
    clip_u(P, S, E, ux, uy);
    reinterpret_cast<double2*>(u)[i] = make_double2(ux, uy);
    status[i] = pack_status(S);
    if (xo) reinterpret_cast<double2*>(xo)[i] = make_double2(S.x0, S.x1);
}

// swarm form: ego e = ego_begin + k with the neighbour indices of cbf_cull_allpairs (reference
// order); ego state (pos, vel), u0 = vel; rows at ws[k * kmax ..]
__global__ void __launch_bounds__(kBlock) k_hocbf_indexed(KP P, HP H, const double2* __restrict__ pos,
                                                          const double2* __restrict__ vel, int ego_begin, int ego_end,
                                                          int kmax, const int32_t* __restrict__ nbr_idx,
                                                          const int32_t* __restrict__ nbr_count,
                                                          double* __restrict__ u, int32_t* __restrict__ status,
                                                          double* __restrict__ xo, double4* __restrict__ ws) {
    const int e = ego_begin + blockIdx.x * kBlock + threadIdx.x;
    if (e >= ego_end) return;
    const long k = e - ego_begin;
    const double2 pe = pos[e], ve = vel[e];
    Ego E;
    ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
    const int m = nbr_count[k];
    double ux = E.u0x, uy = E.u0y;  // no neighbour: filter not run, u0 unclipped (cross_and_rescue.py:153)
    int32_t st = CBF_STATUS_IDLE;
    double x0 = 0.0, x1 = 0.0;
    if (m > kmax) {
        st = CBF_STATUS_NBR_OVERFLOW;
    } else if (m > 0) {
        double4* rows = ws + k * kmax;
        for (int t = 0; t < m; ++t) {
            const int j = nbr_idx[k * kmax + t];
            const double2 pj = pos[j], vj = vel[j];
            rows[t] = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, pj.x, pj.y, vj.x, vj.y, E.u0x, E.u0y);
        }
        StoredRows R{rows, m};
        const Sol S = solve_hocbf(P, E, R);
        clip_u(P, S, E, ux, uy);
        st = pack_status(S);
        x0 = S.x0;
        x1 = S.x1;
    }
    reinterpret_cast<double2*>(u)[k] = make_double2(ux, uy);
    status[k] = st;
    if (xo) reinterpret_cast<double2*>(xo)[k] = make_double2(x0, x1);
}


// Lattice step K4 in HOCBF mode: one lane per cell-sorted slot (owned agents); exact cull over
// the 3x3 cells; hits kept as LDS keys (entity << 32 | slot) in ascending entity order (the
// oracle's reference-order row sequence, independent of the atomic arrival order inside a cell);
// rows recomputed from the cell-sorted state during the solve; clip, Euler, outputs as
// k_lattice_filter.  More than kHocbfCap neighbours: CBF_STATUS_NBR_OVERFLOW, u = u0.
constexpr int kHocbfCap = 24;
// The main HOCBF lattice kernel appends hits unsorted and sorts its <= 8 keys in registers
// (hocbf_sort8) instead of keeping the LDS list sorted by insertion: advance 196.5 vs 219.9 us.
constexpr int kHScan = 6;  // candidates in flight per lane in the HOCBF scan

// Neighbour scan of one ego (slot) over its 3x3 cells; hits go into the ascending-entity key
// list keys[i * ks + lane] (first kHocbfCap of them).  Returns the hit count m.
// SORTED: keep the list sorted by insertion (all kHocbfCap slots); otherwise append the first
// kLdsRows hits unsorted (the main kernel sorts them in registers, hocbf_sort8; egos with more
// hits are queued and rescanned sorted by the wide role).
template <bool SORTED = true>
__device__ __forceinline__ int hocbf_scan(const KP& P, const CellGrid& G, const Ego& E, const double2* __restrict__ spos,
                                          const int32_t* __restrict__ sidx, const int32_t* __restrict__ start,
                                          unsigned long long* keys, int ks, int lane) {
    const int cx = cell_coord(E.r0, G.x0, G.inv_h, G.nx);
    const int cy = cell_coord(E.r1, G.y0, G.inv_h, G.ny);
    const int xa = cx > 0 ? cx - 1 : 0;
    const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
    int m = 0;
    // the three cell-row ranges as one sequence, kHScan candidates (position + entity index)
    // in flight per lane
    int t0[3], t1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int yy = cy + k - 1;
        const bool in = yy >= 0 && yy < G.ny;
        t0[k] = in ? start[yy * G.nx + xa] : 0;
        t1[k] = in ? start[yy * G.nx + xb + 1] : 0;
    }
    const int l0 = t1[0] - t0[0], l01 = l0 + (t1[1] - t0[1]), L = l01 + (t1[2] - t0[2]);
    for (int v = 0; v < L; v += kHScan) {
        double2 pq[kHScan];
        int tq[kHScan], iq[kHScan];
#pragma unroll
        for (int q = 0; q < kHScan; ++q) {
            const int vv = v + q;
            tq[q] = vv < l0 ? t0[0] + vv : (vv < l01 ? t0[1] + (vv - l0) : t0[2] + (vv - l01));
            if (vv < L) {
                pq[q] = spos[tq[q]];
                iq[q] = sidx[tq[q]];
            }
        }
#pragma unroll
        for (int q = 0; q < kHScan; ++q) {
            if (v + q >= L) continue;
            const double q0 = pq[q].x - E.r0, q1 = pq[q].y - E.r1;
            const double sq = q0 * q0 + q1 * q1;
            if (!(sq < P.cull_t && sq > 0)) continue;  // agents only (cross_and_rescue.py:147-150)
            const unsigned long long key = ((unsigned long long)(unsigned)iq[q] << 32) | (unsigned)tq[q];
            if (!SORTED) {
                if (m < kLdsRows) keys[m * ks + lane] = key;
            } else if (m < kHocbfCap) {  // insertion into the sorted list
                int j = m;
                while (j > 0 && keys[(j - 1) * ks + lane] > key) {
                    keys[j * ks + lane] = keys[(j - 1) * ks + lane];
                    --j;
                }
                keys[j * ks + lane] = key;
            }
            ++m;
        }
    }
    return m;
}

// Ascending sort of 8 keys in registers (Batcher odd-even merge network, 19 compare-exchanges;
// keys are unique, so the order equals the insertion-sorted list's).
__device__ __forceinline__ void cas(unsigned long long& a, unsigned long long& b) {
    const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}
__device__ __forceinline__ void hocbf_sort8(unsigned long long (&k)[8]) {
    cas(k[0], k[1]); cas(k[2], k[3]); cas(k[4], k[5]); cas(k[6], k[7]);
    cas(k[0], k[2]); cas(k[1], k[3]); cas(k[4], k[6]); cas(k[5], k[7]);
    cas(k[1], k[2]); cas(k[5], k[6]);
    cas(k[0], k[4]); cas(k[1], k[5]); cas(k[2], k[6]); cas(k[3], k[7]);
    cas(k[2], k[4]); cas(k[3], k[5]);
    cas(k[1], k[2]); cas(k[3], k[4]); cas(k[5], k[6]);
}

// Rows of the m <= cap sorted keys computed once into lds[(3i + c) * ks + lane] (the keys are
// read out first when the row area aliases the key area), then the relaxation loop.  SORT: the
// keys were appended unsorted (cap = 8): sort them in registers first (absent slots = ~0 sort last).
template <int CAP, bool SORT = false>
__device__ __forceinline__ Sol hocbf_solve_lds(const KP& P, const HP& H, const Ego& E, const double2* __restrict__ spos,
                                               const double2* __restrict__ svel, const unsigned long long* keys,
                                               double* rl, int ks, int lane, int m) {
    unsigned long long kr[CAP];
#pragma unroll
    for (int i = 0; i < CAP; ++i) kr[i] = i < m ? keys[i * ks + lane] : ~0ull;
    if constexpr (SORT) {
        static_assert(CAP == 8, "hocbf_sort8 sorts 8 keys");
        hocbf_sort8(kr);
    }
#pragma unroll
    for (int i = 0; i < CAP; ++i) {
        if (i < m) {
            const int sl = (int)(kr[i] & 0xFFFFFFFFull);
            const double2 o = spos[sl], ov = svel[sl];
            const double4 rw = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, o.x, o.y, ov.x, ov.y, E.u0x, E.u0y);
            rl[(3 * i) * ks + lane] = rw.x;
            rl[(3 * i + 1) * ks + lane] = rw.y;
            rl[(3 * i + 2) * ks + lane] = rw.z;
        }
    }
    LdsRows R{rl, ks, lane, m};
    return solve_hocbf(P, E, R);
}

// hocbf_cert for the main kernel, in fp32 on register copies of the <= 8 rows (every loop unrolled,
// no LDS re-reads): the same rows chosen (i the most violated, its two best opposite partners, every
// other row as the third) and the same proof, with the fp32 rounding in the bound -- rows rounded
// to fp32 (relative 2^-24 each, an underflow below 2^-126 absolute), every sum and product of the
// test (a dozen roundings of 2^-24 each), all below 1e-6 mag, so the test asks q < -1e-4 mag (on the
// cfg4 lattice q / mag is about -3e-3).  X0, X1 are fp64 upper bounds rounded up into fp32.
struct CertRowF {
    float a0, a1, b, mg;
};
__device__ __forceinline__ bool cert_triple_f(const CertRowF& I, const CertRowF& J, const CertRowF& K, float lj,
                                              float lk, float X0, float X1) {
    float li = J.a0 * K.a1 - J.a1 * K.a0;  // lj = a_k x a_i, lk = a_i x a_j: the caller's
    const bool pos = li >= 0.0f && lj >= 0.0f && lk >= 0.0f, neg = li <= 0.0f && lj <= 0.0f && lk <= 0.0f;
    li = fabsf(li);  // (one sign for all three when pos || neg: lambda = their magnitudes)
    lj = fabsf(lj);
    lk = fabsf(lk);
    const float sb = (li * I.b + lj * J.b) + lk * K.b;
    const float r0 = (li * I.a0 + lj * J.a0) + lk * K.a0, r1 = (li * I.a1 + lj * J.a1) + lk * K.a1;
    const float mag = (li * I.mg + lj * J.mg) + lk * K.mg;
    const float q = (sb + fabsf(r0) * X0) + fabsf(r1) * X1;
    return (pos || neg) && q < -1e-4f * mag;
}
template <int CAP>
__device__ __forceinline__ bool hocbf_cert_f32(const float (&fa0)[CAP], const float (&fa1)[CAP], const float (&fb)[CAP],
                                               int m, const double (&bb)[4]) {
    if (m < 3) return false;
    double X0d, X1d;
    cert_bounds(bb, X0d, X1d);
    const float X0 = (float)(X0d * (1.0 + 1e-6)), X1 = (float)(X1d * (1.0 + 1e-6));
    int i = 0;
    float bi = fb[0], ai0 = fa0[0], ai1 = fa1[0];
#pragma unroll
    for (int k = 1; k < CAP; ++k) {
        const bool t = k < m && fb[k] < bi;
        bi = t ? fb[k] : bi;
        ai0 = t ? fa0[k] : ai0;
        ai1 = t ? fa1[k] : ai1;
        i = t ? k : i;
    }
    if (!(bi < 0.0f)) return false;
    const float n2 = ai0 * ai0 + ai1 * ai1;
    int j1 = -1, j2 = -1;
    float s1 = INFINITY, s2 = INFINITY;
    CertRowF J1{0.0f, 0.0f, 0.0f, 0.0f}, J2{0.0f, 0.0f, 0.0f, 0.0f};
    float mg[CAP];
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
        mg[k] = 1.0f + fabsf(fb[k]) + fabsf(fa0[k]) * X0 + fabsf(fa1[k]) * X1;
        const float dt = ai0 * fa0[k] + ai1 * fa1[k];
        const float sc = fb[k] * n2 - bi * dt;
        const bool ok = k < m && k != i && dt < 0.0f;
        const bool t1 = ok && sc < s1, t2 = ok && !t1 && sc < s2;
        const CertRowF Kr{fa0[k], fa1[k], fb[k], mg[k]};
        if (t1) {
            s2 = s1;
            j2 = j1;
            J2 = J1;
            s1 = sc;
            j1 = k;
            J1 = Kr;
        }
        if (t2) {
            s2 = sc;
            j2 = k;
            J2 = Kr;
        }
    }
    if (j1 < 0) return false;
    const CertRowF I{ai0, ai1, bi, 1.0f + fabsf(bi) + fabsf(ai0) * X0 + fabsf(ai1) * X1};
    const float lk1 = ai0 * J1.a1 - ai1 * J1.a0, lk2 = ai0 * J2.a1 - ai1 * J2.a0;
    bool cert = false;
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
        const CertRowF K{fa0[k], fa1[k], fb[k], mg[k]};
        const float lj = K.a0 * ai1 - K.a1 * ai0;  // a_k x a_i
        const bool in = k < m && k != i;
        cert = cert || (in && k != j1 && cert_triple_f(I, J1, K, lj, lk1, X0, X1));
        if (CBF_HOCBF_CERT_J > 1) cert = cert || (in && j2 >= 0 && k != j2 && cert_triple_f(I, J2, K, lj, lk2, X0, X1));
    }
    return cert;
}

// The main lattice kernel's part of the solve (CBF_HOCBF_CERT): the QPs settled without one
// Seidel event.  After the box phase (solve_rows' first part; a failure there is solve_hocbf's
// BOX_INFEASIBLE), the first pass has no event exactly when every row holds at its point xb, and
// then returns xb (OPTIMAL); when hocbf_cert_f32 proves the unrelaxed rows infeasible (so the first
// pass fails at a row) and a relaxation is allowed, the second pass likewise returns xb (RELAXED,
// one relaxation) when every row + 1 holds there.  Everything else -- about one ego in ten at cfg4
// -- goes whole, with its sorted neighbour slots, to k_lattice_filter_hocbf_hard: a lane-per-ego
// loop runs as many Seidel passes as its slowest lane needs, so the egos that take events are
// gathered into full waves of their own.  True with S set when settled; nb: the row order's slots.
struct HocbfHardRec {
    int slot, m;
    int nb[8];
};
constexpr int kHardQ2 = 16;  // the hard queue's counters: word 16 of each of the header's queue lines
// its records: after the wide queue's slots in the queue area (CellWs::qrec holds kSubQ qcap
// HardRecs of 104 B; slots 4 B + these 40 B per entry fit)
__device__ __host__ inline HocbfHardRec* hocbf_hard_rec(int32_t* qslot, long qcap) {
    return reinterpret_cast<HocbfHardRec*>(reinterpret_cast<char*>(qslot) +
                                            ((4 * (size_t)kSubQ * qcap + 255) & ~(size_t)255));
}
static_assert(sizeof(HocbfHardRec) + 4 <= sizeof(HardRec), "the queue area holds both HOCBF queues");
__device__ __forceinline__ bool hocbf_settle(const KP& P, const HP& H, const Ego& E, const double2* __restrict__ spos,
                                             const double2* __restrict__ svel, const unsigned long long* keys, int ks,
                                             int lane, int m, Sol& S, int (&nb)[kLdsRows]) {
    S.status = CBF_STATUS_OPTIMAL;
    S.iters = 0;
    S.x0 = S.x1 = 0.0;
    S.viol = 0.0;
    const Box B = box_rhs(P, E);
    const double bb[4] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7])};
    double xb0, xb1;
    if (box_phase(bb, xb0, xb1) >= 0) {  // solve_hocbf's first pass fails in its box phase
        S.status = CBF_STATUS_BOX_INFEASIBLE;
        return true;
    }
    unsigned long long kr[kLdsRows];
#pragma unroll
    for (int i = 0; i < kLdsRows; ++i) kr[i] = i < m ? keys[i * ks + lane] : ~0ull;
    hocbf_sort8(kr);
    float fa0[kLdsRows], fa1[kLdsRows], fb[kLdsRows];  // the certificate's fp32 copies
    bool ok0 = true, ok1 = true;
#pragma unroll
    for (int i = 0; i < kLdsRows; ++i) {
        fa0[i] = fa1[i] = fb[i] = 0.0f;
        nb[i] = (int)(kr[i] & 0xFFFFFFFFull);
        if (i < m) {
            const double2 o = spos[nb[i]], ov = svel[nb[i]];
            const double4 rw = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, o.x, o.y, ov.x, ov.y, E.u0x, E.u0y);
            ok0 = ok0 && feas(rw.x, rw.y, rw.z, xb0, xb1);
            ok1 = ok1 && feas(rw.x, rw.y, rw.z + 1.0, xb0, xb1);  // (the relaxed row: cbf.py:85-87)
            fa0[i] = (float)rw.x;
            fa1[i] = (float)rw.y;
            fb[i] = (float)rw.z;
        }
    }
    if (ok0) {
        S.x0 = xb0;
        S.x1 = xb1;
        return true;
    }
#if CBF_DIAG_CERT_TRUE  // diagnostic only (wrong statuses): the certificate taken as given
    if (ok1 && P.relax_cap >= 1) {
#else
    if (ok1 && P.relax_cap >= 1 && hocbf_cert_f32<kLdsRows>(fa0, fa1, fb, m, bb)) {
#endif
        S.status = CBF_STATUS_RELAXED;
        S.iters = 1;
        S.x0 = xb0;
        S.x1 = xb1;
        return true;
    }
    return false;
}

// Outputs of an owned ego (clip, Euler, status, count) and its guard extents.
__device__ __forceinline__ void hocbf_finish(const KP& P, const Sol* S, const Ego& E, int m, int W, int row_begin,
                                             int row_end, int r, int c, double T, double2* __restrict__ pos_out,
                                             double2* __restrict__ u, int32_t* __restrict__ status,
                                             int32_t* __restrict__ cnt, int guard_rows, double& e0, double& e1,
                                             double& e2, double& e3) {
    double ux = E.u0x, uy = E.u0y;  // no neighbour: filter not run, u0 unclipped
    int32_t st = m > kHocbfCap ? CBF_STATUS_NBR_OVERFLOW : CBF_STATUS_IDLE;
    if (S) {
        clip_u(P, *S, E, ux, uy);
        st = pack_status(*S);
    }
    const long k = (long)(r - row_begin) * W + c;
    const double2 pn = make_double2(E.r0 + T * ux, E.r1 + T * uy);
    pos_out[k] = pn;
    u[k] = make_double2(ux, uy);
    status[k] = st;
    if (cnt) cnt[k] = m;
    ext_accumulate(r, row_begin, row_end, guard_rows, pn.y, e0, e1, e2, e3);
}

// Lattice step K4 in HOCBF mode: one lane per cell-sorted slot (owned agents); exact cull over
// the 3x3 cells; hits kept as LDS keys (entity << 32 | slot) in ascending entity order (the
// oracle's reference-order row sequence, independent of the atomic arrival order inside a cell);
// the QP settled here when it needs no Seidel event (hocbf_settle, CBF_HOCBF_CERT), else queued
// whole for the hard role of k_lattice_filter_hocbf_rest (without CBF_HOCBF_CERT: the rows in LDS and
// the full solve here); clip, Euler, outputs as k_lattice_filter.  Egos with more than kLdsRows
// neighbours are queued (their slot, hardq) for the wide role, so the long tail does not hold
// whole waves; more than kHocbfCap: CBF_STATUS_NBR_OVERFLOW, u = u0.
__global__ void __launch_bounds__(kBlock) k_lattice_filter_hocbf(
    KP P, HP H, CellGrid G, int W, int row_begin, int row_end, int win_row0, long nwin, long ncell,
    const double2* __restrict__ spos, const double2* __restrict__ svel, const int32_t* __restrict__ sidx,
    const int32_t* __restrict__ start, double T, double2* __restrict__ pos_out, double2* __restrict__ u,
    int32_t* __restrict__ status, int32_t* __restrict__ cnt, int guard_rows, double* __restrict__ ext_part,
    unsigned long long* __restrict__ solves, int32_t* __restrict__ hardq, int32_t* __restrict__ qslot, long qcap,
    const int32_t* __restrict__ sctl) {
#if CBF_HOCBF_CERT
    __shared__ unsigned long long keys[kLdsRows * kBlock];
#else
    __shared__ unsigned long long keys[kHocbfCap * kBlock];  // the keys, then the rows (3 doubles each)
#endif
    const int bx = xcd_block();
    const int slot = bx * kBlock + threadIdx.x;
    if (sctl[2] != 0) {  // unusable cell list (build_begin / scan timeout): touch none of it
        lattice_error_tail(W, row_begin, row_end, win_row0, nwin, slot, u, status, cnt, solves, ext_part,
                           (long)bx * (kBlock / 64) + (threadIdx.x >> 6), hardq);
        return;
    }
    const int total = start[ncell];
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    bool solved = false;
    if (slot < total) {
        const int w = sidx[slot];
        const int r = win_row0 + w / W, c = w % W;
        if (r >= row_begin && r < row_end) {
            const double2 pe = spos[slot], ve = svel[slot];
            Ego E;
            ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
            const int m = hocbf_scan<false>(P, G, E, spos, sidx, start, keys, kBlock, threadIdx.x);
            E.count = m;
            if (m > kLdsRows && m <= kHocbfCap) {
                const long rec = subq_append(hardq, bx % kSubQ, qcap);
                if (rec >= 0) qslot[rec] = slot;  // (always: the queue holds every agent)
            } else if (CBF_HOCBF_CERT && m > 0 && m <= kLdsRows) {
                Sol S;
                int nb[kLdsRows];
                if (hocbf_settle(P, H, E, spos, svel, keys, kBlock, threadIdx.x, m, S, nb)) {
                    solved = true;
                    hocbf_finish(P, &S, E, m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows,
                                 e0, e1, e2, e3);
                } else {  // the Seidel events: k_lattice_filter_hocbf_hard
                    const long rec = subq_append(hardq + kHardQ2, bx % kSubQ, qcap);
                    if (rec >= 0) {  // (always: the queue holds every agent)
                        HocbfHardRec& h = hocbf_hard_rec(qslot, qcap)[rec];
                        h.slot = slot;
                        h.m = m;
#pragma unroll
                        for (int i = 0; i < kLdsRows; ++i) h.nb[i] = nb[i];
                    }
                }
            } else if (m > 0 && m <= kLdsRows) {
                const Sol S = hocbf_solve_lds<kLdsRows, true>(P, H, E, spos, svel, keys, reinterpret_cast<double*>(keys),
                                                        kBlock, threadIdx.x, m);
                solved = true;
                hocbf_finish(P, &S, E, m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows, e0,
                             e1, e2, e3);
            } else {
                hocbf_finish(P, nullptr, E, m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows,
                             e0, e1, e2, e3);
            }
        }
    }
    if (solves) {
        const unsigned long long mk = __ballot(solved);
        if ((threadIdx.x & 63) == 0 && mk)
            atomicAdd(&solves[16 * stat_slot(bx * (kBlock / 64) + (threadIdx.x >> 6))],
                      (unsigned long long)__popcll(mk));
    }
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, (long)bx * (kBlock / 64) + (threadIdx.x >> 6));
}

// ---- the wide egos (kLdsRows < m <= kHocbfCap, and those the main kernel's one pass left unsolved):
// one ego per wave, its rows across the lanes ----
// A lane-per-ego solve of such an ego is a chain of O(m^2) dependent row steps (up to 24 rows,
// ~90 % of the QPs solved twice for the +1 relaxation); here lane i holds row i, so the feasibility
// tests of every row run at once and only the interval fold of solve_rows stays serial.

// lane l's double, read wave-uniformly (l uniform)
__device__ __forceinline__ double rdl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __hiloint2double(hi, lo);
}

// Interval::add with the row's ad and r already formed (the same expressions, in the lane)
__device__ __forceinline__ void interval_add(Interval& I, double ad, double r) {
    if (ad > 0) {
        if (!I.has_hi || r * I.ah < I.rh * ad) {
            I.rh = r;
            I.ah = ad;
        }
        I.has_hi = true;
    } else if (ad < 0) {
        if (!I.has_lo || r * I.al > I.rl * ad) {
            I.rl = r;
            I.al = ad;
        }
        I.has_lo = true;
    }
}

// solve_rows over the 4 box planes and the m rows held one per lane (a0, a1, b of lane i = row i):
// the same events in the same order with the same arithmetic.  The next event is the first row
// at or after i infeasible at the current x (one ballot: the sequential loop skips exactly the
// feasible rows before it); its interval folds the box planes, then rows 0 .. i-1 in row order
// (their ad and r formed in every lane at once, the fold itself serial, as the comparisons are);
// the check after the step is one ballot over rows 0 .. i.
__device__ __forceinline__ int solve_rows_wave(const double (&bb)[4], double a0, double a1, double b, int m, int lane,
                                               double& xo0, double& xo1) {
    const double ba0[4] = {1.0, 0.0, -1.0, 0.0}, ba1[4] = {0.0, 1.0, 0.0, -1.0};
    double x0 = 0.0, x1 = 0.0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {  // box planes: solve_rows' own code (wave-uniform)
        if (feas(ba0[h], ba1[h], bb[h], x0, x1)) continue;
        const double n2 = ba0[h] * ba0[h] + ba1[h] * ba1[h];
        const double t = bb[h] / n2;
        const double p0 = t * ba0[h], p1 = t * ba1[h];
        const double d0 = -ba1[h], d1 = ba0[h];
        Interval I;
#pragma unroll
        for (int j = 0; j < h; ++j) I.add(ba0[j], ba1[j], bb[j], d0, d1, p0, p1);
        const double s = I.clamp0();
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j <= h; ++j) ok = ok && feas(ba0[j], ba1[j], bb[j], x0, x1);
        if (!ok) return h;
    }
    const bool mine = lane < m;
    int i = 0;
    for (;;) {
        const unsigned long long bad = __ballot(mine && lane >= i && !feas(a0, a1, b, x0, x1));
        if (!bad) break;
        const int e = __ffsll((long long)bad) - 1;
        const double ea0 = rdl(a0, e), ea1 = rdl(a1, e), eb = rdl(b, e);
        const double n2 = ea0 * ea0 + ea1 * ea1;
        if (!(n2 > 0)) return 4 + e;
        const double t = eb / n2;
        const double p0 = t * ea0, p1 = t * ea1;
        const double d0 = -ea1, d1 = ea0;
        Interval I;
#pragma unroll
        for (int j = 0; j < 4; ++j) I.add(ba0[j], ba1[j], bb[j], d0, d1, p0, p1);
        const double ad = a0 * d0 + a1 * d1;
        const double r = b - (a0 * p0 + a1 * p1);
        for (int j = 0; j < e; ++j) interval_add(I, rdl(ad, j), rdl(r, j));
        const double s = I.clamp0();
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok = ok && feas(ba0[j], ba1[j], bb[j], x0, x1);
        if (!ok) return 4 + e;
        if (__ballot(mine && lane <= e && !feas(a0, a1, b, x0, x1))) return 4 + e;
        i = e + 1;
    }
    xo0 = x0;
    xo1 = x1;
    return -1;
}

// hocbf_cert over the rows held one per lane (lane t < m: row t): i and j found by wave
// reductions, every lane's row tried as the third; the same test and proof (any i, j, k do).
__device__ __forceinline__ bool hocbf_cert_wave(double a0, double a1, double b, int m, int lane,
                                                const double (&bb)[4]) {
    if (m < 3) return false;
    const bool mine = lane < m;
    const double bmin = __ockl_wfred_min_f64(mine ? b : INFINITY);
    if (!(bmin < 0.0)) return false;
    const unsigned long long mi_ = __ballot(mine && b == bmin);
    const int i = __ffsll((long long)mi_) - 1;
    const double ai0 = rdl(a0, i), ai1 = rdl(a1, i), bi = rdl(b, i);
    const double dt = ai0 * a0 + ai1 * a1;
    const double sc = b * (ai0 * ai0 + ai1 * ai1) - bi * dt;
    const bool cand = mine && lane != i && dt < 0.0;
    const double smin = __ockl_wfred_min_f64(cand ? sc : INFINITY);
    const unsigned long long mj_ = __ballot(cand && sc == smin);
    if (!mj_) return false;
    const int j = __ffsll((long long)mj_) - 1;
    double X0, X1;
    cert_bounds(bb, X0, X1);
    const CertRow I = cert_row(ai0, ai1, bi, X0, X1), J = cert_row(rdl(a0, j), rdl(a1, j), rdl(b, j), X0, X1);
    const CertRow K = cert_row(a0, a1, b, X0, X1);
    return __ballot(mine && lane != i && lane != j && cert_triple(I, J, K, X0, X1)) != 0;
}

// solve_hocbf over the lanes' rows: +1 relaxation of every row while infeasible (CBF_HOCBF_CERT:
// a first pass hocbf_cert_wave proves infeasible is skipped, as solve_hocbf does)
__device__ __forceinline__ Sol solve_hocbf_wave(const KP& P, const Ego& E, double a0, double a1, double b, int m,
                                                int lane) {
    const Box B = box_rhs(P, E);
    const double bb[4] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7])};
    Sol S;
    S.status = CBF_STATUS_OPTIMAL;
    S.iters = 0;
    S.x0 = S.x1 = 0.0;
    S.viol = 0.0;
    if (CBF_HOCBF_CERT && P.relax_cap >= 1) {
        double xb0, xb1;
        if (box_phase(bb, xb0, xb1) < 0 && hocbf_cert_wave(a0, a1, b, m, lane, bb)) {
            b = b + 1.0;  // cbf.py:85-87
            S.iters = 1;
            S.status = CBF_STATUS_RELAXED;
        }
    }
    for (;;) {
        const int fail = solve_rows_wave(bb, a0, a1, b, m, lane, S.x0, S.x1);
        if (fail < 0) break;
        if (fail < 4) {
            S.status = CBF_STATUS_BOX_INFEASIBLE;
            S.x0 = S.x1 = 0.0;
            break;
        }
        if (S.iters >= P.relax_cap) {
            S.status = CBF_STATUS_RELAX_CAP;
            S.x0 = S.x1 = 0.0;
            break;
        }
        b = b + 1.0;  // cbf.py:85-87
        S.iters++;
        S.status = CBF_STATUS_RELAXED;
    }
    return S;
}

// 64-bit keys sorted ascending across the wave (bitonic network; lane i gets the i-th smallest)
__device__ __forceinline__ unsigned long long wave_sort64(unsigned long long key, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const unsigned lo = __shfl_xor((unsigned)key, j, 64), hi = __shfl_xor((unsigned)(key >> 32), j, 64);
            const unsigned long long o = ((unsigned long long)hi << 32) | lo;
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            key = keep_min ? (o < key ? o : key) : (o > key ? o : key);
        }
    return key;
}

// The queued egos, one per 64-lane block (sub-queue q's entries k, k + nwork, ... for its k-th
// working block): the 3x3-cell candidates tested one per lane, the hits' keys (entity << 32 |
// slot) sorted across the lanes into the reference's row order, lane i forms row i, then the
// wave's solve.  The same neighbour set, rows and solve as hocbf_scan + hocbf_solve_lds, bit for
// bit.  More candidates than lanes are taken 64 at a time into LDS.
// solve_rows for rows staged in LDS (LdsRows) with the loops over earlier rows unrolled over all
// CAP slots and predicated (j < i), so that each event's row loads issue together instead of one
// guarded round trip per row; the same events, arithmetic and order.  The checks after an event
// return 4 + i whichever plane fails first, so they are one conjunction.
template <int CAP>
__device__ __forceinline__ int solve_rows_batched(const double (&bb)[4], const LdsRows& R, double& xo0,
                                                  double& xo1) {
    const double ba0[4] = {1.0, 0.0, -1.0, 0.0}, ba1[4] = {0.0, 1.0, 0.0, -1.0};
    double x0, x1;
    const int hb = box_phase(bb, x0, x1);
    if (hb >= 0) return hb;
    for (int i = 0; i < R.m; ++i) {
        double a0, a1, b;
        R.row(i, a0, a1, b);
        if (feas(a0, a1, b, x0, x1)) continue;
        const double n2 = a0 * a0 + a1 * a1;
        if (!(n2 > 0)) return 4 + i;
        const double t = b / n2;
        const double p0 = t * a0, p1 = t * a1;
        const double d0 = -a1, d1 = a0;
        Interval I;
#pragma unroll
        for (int j = 0; j < 4; ++j) I.add(ba0[j], ba1[j], bb[j], d0, d1, p0, p1);
#pragma unroll
        for (int j = 0; j < CAP; ++j) {
            double c0, c1, e;
            R.row(j, c0, c1, e);
            if (j < i) I.add(c0, c1, e, d0, d1, p0, p1);
        }
        const double s = I.clamp0();
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok = ok & feas(ba0[j], ba1[j], bb[j], x0, x1);
#pragma unroll
        for (int j = 0; j < CAP; ++j) {
            double c0, c1, e;
            R.row(j, c0, c1, e);
            ok = ok & (j > i || feas(c0, c1, e, x0, x1));
        }
        if (!ok) return 4 + i;
    }
    xo0 = x0;
    xo1 = x1;
    return -1;
}
// solve_hocbf over solve_rows_batched
__device__ __forceinline__ Sol solve_hocbf_batched(const KP& P, const Ego& E, LdsRows& R) {
    const Box B = box_rhs(P, E);
    const double bb[4] = {pmin(B.S[0], B.S[4]), pmin(B.S[1], B.S[6]), pmin(B.S[2], B.S[5]), pmin(B.S[3], B.S[7])};
    Sol S;
    S.status = CBF_STATUS_OPTIMAL;
    S.iters = 0;
    S.x0 = S.x1 = 0.0;
    S.viol = 0.0;
    for (;;) {  // oracle/cbf_oracle.c:solve_hocbf
        const int fail = solve_rows_batched<kLdsRows>(bb, R, S.x0, S.x1);
        if (fail < 0) break;
        if (fail < 4) {
            S.status = CBF_STATUS_BOX_INFEASIBLE;
            S.x0 = S.x1 = 0.0;
            break;
        }
        if (S.iters >= P.relax_cap) {
            S.status = CBF_STATUS_RELAX_CAP;
            S.x0 = S.x1 = 0.0;
            break;
        }
        R.relax();
        S.iters++;
        S.status = CBF_STATUS_RELAXED;
    }
    return S;
}

// blocks per sub-queue of the hard role: ~10 % of the egos at cfg4 (~2 k per sub-queue) in one
// round of lanes
#ifndef CBF_HOCBF_HARD_PER_Q
#define CBF_HOCBF_HARD_PER_Q 64
#endif
constexpr int kHocbfHardPerQ = CBF_HOCBF_HARD_PER_Q;
static_assert(kHocbfHardPerQ <= 128, "lattice_ext_bytes reserves 128 blocks per sub-queue");

// The egos hocbf_settle left (CBF_HOCBF_CERT): solve_hocbf whole, one lane per ego, rows formed
// from the queued neighbour slots into LDS, the sub-queue drained in full waves as drain_subq does
// -- the main kernel's own solve (hocbf_solve_lds), on waves made only of such egos.
// (block bid of the hard role; rl: 3 kLdsRows 64 doubles of LDS)
__device__ __forceinline__ void hocbf_hard_block(
    int bid, double* rl, const KP& P, const HP& H, int W, int row_begin, int row_end, int win_row0,
    const double2* __restrict__ spos, const double2* __restrict__ svel, const int32_t* __restrict__ sidx, double T,
    double2* __restrict__ pos_out, double2* __restrict__ u, int32_t* __restrict__ status, int32_t* __restrict__ cnt,
    int guard_rows, double* __restrict__ ext_part, unsigned long long* __restrict__ solves,
    int32_t* __restrict__ hardq, int32_t* __restrict__ qslot, long qcap) {
    const int lane = threadIdx.x;
    const HocbfHardRec* __restrict__ hrec = hocbf_hard_rec(qslot, qcap);
    int32_t* __restrict__ hq = hardq + kHardQ2;
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    int ns = 0;
    // drain_subq for block bid
    const int q = bid % kSubQ, kb = bid / kSubQ;
    const int nq0 = hq[32 * (1 + q)];
    const int nq = nq0 < qcap ? nq0 : (int)qcap;
    const int need = (nq + 63) / 64;
    const int nwork = need < kHocbfHardPerQ ? need : kHocbfHardPerQ;
    if (kb >= nwork) return;
    int done = 0;
    if (lane == 0) done = atomicAdd(&hq[32 * (1 + kSubQ + q)], 1);
    for (int i = kb * 64 + lane; i < nq; i += nwork * 64) {
        const HocbfHardRec h = hrec[(long)q * qcap + i];
        const int w = sidx[h.slot];
        const int r = win_row0 + w / W, c = w % W;
        const double2 pe = spos[h.slot], ve = svel[h.slot];
        Ego E;
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
        E.count = h.m;
#pragma unroll
        for (int k = 0; k < kLdsRows; ++k) {
            if (k < h.m) {
                const double2 o = spos[h.nb[k]], ov = svel[h.nb[k]];
                const double4 rw = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, o.x, o.y, ov.x, ov.y, E.u0x, E.u0y);
                rl[(3 * k) * 64 + lane] = rw.x;
                rl[(3 * k + 1) * 64 + lane] = rw.y;
                rl[(3 * k + 2) * 64 + lane] = rw.z;
            }
        }
        LdsRows R{rl, 64, lane, h.m};
#if CBF_HOCBF_HARD_BATCHED
        const Sol S = solve_hocbf_batched(P, E, R);
#else
        const Sol S = solve_hocbf(P, E, R);
#endif
        hocbf_finish(P, &S, E, h.m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows, e0, e1, e2,
                     e3);
        ++ns;
    }
    if (lane == 0 && done == nwork - 1) {  // the last working block empties the sub-queue
        hq[32 * (1 + q)] = 0;
        hq[32 * (1 + kSubQ + q)] = 0;
    }
    if (solves) {
        int tot = ns;
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd(&solves[16 * stat_slot(bid)], (unsigned long long)tot);
    }
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, bid);
}

// (block bid of the wide role; hits: kHocbfCap + 64 words of LDS)
__device__ __forceinline__ void hocbf_wide_block(
    int bid, unsigned long long* hits, const KP& P, const HP& H, const CellGrid& G, int W, int row_begin,
    int row_end, int win_row0, const double2* __restrict__ spos, const double2* __restrict__ svel,
    const int32_t* __restrict__ sidx, const int32_t* __restrict__ start, double T, double2* __restrict__ pos_out,
    double2* __restrict__ u, int32_t* __restrict__ status, int32_t* __restrict__ cnt, int guard_rows,
    double* __restrict__ ext_part, unsigned long long* __restrict__ solves, int32_t* __restrict__ hardq,
    const int32_t* __restrict__ qslot, long qcap) {
    const int lane = threadIdx.x;
    double e0 = INFINITY, e1 = -INFINITY, e2 = -INFINITY, e3 = INFINITY;
    int ns = 0;
    const int q = bid % kSubQ, k = bid / kSubQ;
    const int nq0 = hardq[32 * (1 + q)];
    const int nq = nq0 < qcap ? nq0 : (int)qcap;  // (a full sub-queue's counter runs past qcap: subq_append)
    const int nwork = nq < kWidePerQ ? nq : kWidePerQ;
    if (k >= nwork) return;
    int done = 0;
    if (lane == 0) done = atomicAdd(&hardq[32 * (1 + kSubQ + q)], 1);
    for (int it = k; it < nq; it += nwork) {
        const int slot = qslot[(long)q * qcap + it];
        const int w = sidx[slot];
        const int r = win_row0 + w / W, c = w % W;
        const double2 pe = spos[slot], ve = svel[slot];
        Ego E;
        ego_init(P, E, pe.x, pe.y, ve.x, ve.y, ve.x, ve.y);
        // candidates: the three cell-row ranges of hocbf_scan as one sequence, a lane each
        const int cx = cell_coord(E.r0, G.x0, G.inv_h, G.nx);
        const int cy = cell_coord(E.r1, G.y0, G.inv_h, G.ny);
        const int xa = cx > 0 ? cx - 1 : 0;
        const int xb = cx < G.nx - 1 ? cx + 1 : G.nx - 1;
        int t0[3], t1[3];
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
            const int yy = cy + kk - 1;
            const bool in = yy >= 0 && yy < G.ny;
            t0[kk] = in ? start[yy * G.nx + xa] : 0;
            t1[kk] = in ? start[yy * G.nx + xb + 1] : 0;
        }
        const int l0 = t1[0] - t0[0], l01 = l0 + (t1[1] - t0[1]), L = l01 + (t1[2] - t0[2]);
        int m = 0;
        for (int v0 = 0; v0 < L; v0 += 64) {
            const int v = v0 + lane;
            bool hit = false;
            unsigned long long key = 0;
            if (v < L) {
                const int t = v < l0 ? t0[0] + v : (v < l01 ? t0[1] + (v - l0) : t0[2] + (v - l01));
                const double2 pq = spos[t];
                const double q0 = pq.x - E.r0, q1 = pq.y - E.r1;
                const double sq = q0 * q0 + q1 * q1;
                hit = sq < P.cull_t && sq > 0;  // agents only (cross_and_rescue.py:147-150)
                key = ((unsigned long long)(unsigned)sidx[t] << 32) | (unsigned)t;
            }
            const unsigned long long mk = __ballot(hit);
            const int at = m + __popcll(mk & ((1ull << lane) - 1ull));
            if (hit && at < kHocbfCap + 64) hits[at] = key;
            m += __popcll(mk);
        }
        __syncthreads();  // (the block is this one wave: orders the hit list's writes before its reads)
        E.count = m;
        if (m > kHocbfCap) {  // (not queued by the main kernel; reported as it would be)
            if (lane == 0)
                hocbf_finish(P, nullptr, E, m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows,
                             e0, e1, e2, e3);
            continue;
        }
        // the reference's row order (ascending entity) across the lanes, then lane i's row
        const unsigned long long key = wave_sort64(lane < m ? hits[lane] : ~0ull, lane);
        double a0 = 0.0, a1 = 0.0, b = 0.0;
        if (lane < m) {
            const int sl = (int)(key & 0xFFFFFFFFull);
            const double2 o = spos[sl], ov = svel[sl];
            const double4 rw = hocbf_row(P, H, E.r0, E.r1, E.r2, E.r3, o.x, o.y, ov.x, ov.y, E.u0x, E.u0y);
            a0 = rw.x;
            a1 = rw.y;
            b = rw.z;
        }
        const Sol S = solve_hocbf_wave(P, E, a0, a1, b, m, lane);
        if (lane == 0) {
            ++ns;
            hocbf_finish(P, &S, E, m, W, row_begin, row_end, r, c, T, pos_out, u, status, cnt, guard_rows, e0, e1,
                         e2, e3);
        }
    }
    if (lane == 0 && done == nwork - 1) {  // the last working block empties the sub-queue (drain_subq)
        hardq[32 * (1 + q)] = 0;
        hardq[32 * (1 + kSubQ + q)] = 0;
    }
    if (solves && lane == 0 && ns) atomicAdd(&solves[16 * stat_slot(bid)], (unsigned long long)ns);
    if (ext_part) wave_extents(e0, e1, e2, e3, ext_part, bid);
}

__global__ void __launch_bounds__(64) k_lattice_filter_hocbf_wide(
    KP P, HP H, CellGrid G, int W, int row_begin, int row_end, int win_row0, const double2* __restrict__ spos,
    const double2* __restrict__ svel, const int32_t* __restrict__ sidx, const int32_t* __restrict__ start, double T,
    double2* __restrict__ pos_out, double2* __restrict__ u, int32_t* __restrict__ status, int32_t* __restrict__ cnt,
    int guard_rows, double* __restrict__ ext_part, unsigned long long* __restrict__ solves,
    int32_t* __restrict__ hardq, const int32_t* __restrict__ qslot, long qcap) {
    __shared__ unsigned long long hits[kHocbfCap + 64];
    hocbf_wide_block(blockIdx.x, hits, P, H, G, W, row_begin, row_end, win_row0, spos, svel, sidx, start, T, pos_out,
                     u, status, cnt, guard_rows, ext_part, solves, hardq, qslot, qcap);
}

// The rest of a HOCBF advance in one launch (CBF_HOCBF_CERT): blocks [0, hh) drain the hard queue
// (hocbf_hard_block), the others the wide queue (hocbf_wide_block) -- two latency-bound sets of
// chains side by side instead of one launch after the other.  Extents records: the hard blocks',
// then the wide blocks'.
__global__ void __launch_bounds__(64) k_lattice_filter_hocbf_rest(
    KP P, HP H, CellGrid G, int W, int row_begin, int row_end, int win_row0, const double2* __restrict__ spos,
    const double2* __restrict__ svel, const int32_t* __restrict__ sidx, const int32_t* __restrict__ start, double T,
    double2* __restrict__ pos_out, double2* __restrict__ u, int32_t* __restrict__ status, int32_t* __restrict__ cnt,
    int guard_rows, double* __restrict__ ext_part, unsigned long long* __restrict__ solves,
    int32_t* __restrict__ hardq, int32_t* __restrict__ qslot, long qcap, int hh) {
    __shared__ double lds[3 * kLdsRows * 64];
    static_assert(sizeof(lds) >= 8 * (kHocbfCap + 64), "the wide role's hit list fits the hard role's rows");
    const int b = blockIdx.x;
    if (b < hh)
        hocbf_hard_block(b, lds, P, H, W, row_begin, row_end, win_row0, spos, svel, sidx, T, pos_out, u, status, cnt,
                         guard_rows, ext_part, solves, hardq, qslot, qcap);
    else
        hocbf_wide_block(b - hh, reinterpret_cast<unsigned long long*>(lds), P, H, G, W, row_begin, row_end, win_row0,
                         spos, svel, sidx, start, T, pos_out, u, status, cnt, guard_rows,
                         ext_part ? ext_part + 4l * hh : nullptr, solves, hardq, qslot, qcap);
}

inline int nblocks(long n) { return (int)((n + kBlock - 1) / kBlock); }

inline HP make_hp(const cbf_hocbf* h) {
    HP o;
    o.a_sum = h->alpha1 + h->alpha2;
    o.a_prod = h->alpha1 * h->alpha2;
    return o;
}

}  // namespace

extern "C" size_t cbf_hocbf_workspace_size(int64_t rows) { return rows > 0 ? 32 * (size_t)rows : 32; }

extern "C" int cbf_get_safe_control_batch_hocbf(const cbf_params* p, const cbf_hocbf* hp, int32_t n_ego,
                                                const double* robot_state, const double* u0, const int32_t* nbr_off,
                                                const double* obs_states, double* u, int32_t* status, double* x_out,
                                                void* workspace, size_t workspace_bytes, void* stream) {
    if (!p || !hp || n_ego < 0) return CBF_EINVAL;
    if (n_ego == 0) return 0;
    if (!robot_state || !u0 || !nbr_off || !u || !status || !workspace) return CBF_EINVAL;
    // the row count lives on the device (nbr_off[n_ego]): the caller sizes the workspace for it
    if (workspace_bytes < 32) return CBF_EINVAL;
    hipLaunchKernelGGL(k_hocbf_batch, dim3(nblocks(n_ego)), dim3(kBlock), 0, (hipStream_t)stream, make_kp(p),
                       make_hp(hp), n_ego, robot_state, u0, nbr_off, obs_states, u, status, x_out,
                       reinterpret_cast<double4*>(workspace));
    return (int)hipGetLastError();
}

extern "C" int cbf_filter_indexed_hocbf(const cbf_params* p, const cbf_hocbf* hp, int32_t n, const double* pos,
                                        const double* vel, int32_t ego_begin, int32_t ego_end, int32_t kmax,
                                        const int32_t* nbr_idx, const int32_t* nbr_count, double* u, int32_t* status,
                                        double* x_out, void* workspace, size_t workspace_bytes, void* stream) {
    if (!p || !hp || n < 0 || ego_begin < 0 || ego_end > n || ego_begin > ego_end || kmax < 0) return CBF_EINVAL;
    const long ne = ego_end - ego_begin;
    if (ne == 0) return 0;
    if (!pos || !vel || !nbr_count || !u || !status || (kmax > 0 && (!nbr_idx || !workspace))) return CBF_EINVAL;
    if (kmax > 0 && workspace_bytes < cbf_hocbf_workspace_size(ne * kmax)) return CBF_EINVAL;
    hipLaunchKernelGGL(k_hocbf_indexed, dim3(nblocks(ne)), dim3(kBlock), 0, (hipStream_t)stream, make_kp(p),
                       make_hp(hp), reinterpret_cast<const double2*>(pos), reinterpret_cast<const double2*>(vel),
                       ego_begin, ego_end, kmax, nbr_idx, nbr_count, u, status, x_out,
                       reinterpret_cast<double4*>(workspace));
    return (int)hipGetLastError();
}

extern "C" int cbf_lattice_advance_hocbf(const cbf_params* p, const cbf_hocbf* hp, const cbf_grid* grid, int32_t W,
                                         int32_t H, int32_t row_begin, int32_t row_end, int32_t win_row0,
                                         int32_t win_rows, const double* pos, double T, double* pos_out, double* u,
                                         int32_t* status, int32_t* nbr_count, int32_t guard_rows, double* extents,
                                         uint64_t* solves, void* workspace, size_t workspace_bytes, void* stream) {
    if (!hp) return CBF_EINVAL;
    int rc = check_lattice(p, grid, W, H, row_begin, row_end, win_row0, win_rows, pos, workspace, workspace_bytes);
    if (rc) return rc;
    if (!pos_out || !u || !status) return CBF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const long n = (long)W * win_rows;
    const CellGrid G = make_grid(grid);
    CellWs Wk(workspace, n, (long)G.nx * G.ny);
    double* ext_part = extents ? (double*)((char*)workspace + CellWs::bytes(n, Wk.ncell)) : nullptr;
    const int nb = nblocks(n);
    hipLaunchKernelGGL(k_lattice_filter_hocbf, dim3(nb), dim3(kBlock), 0, s, make_kp(p), make_hp(hp), G, W, row_begin,
                       row_end, win_row0, n, Wk.ncell, Wk.spos, Wk.svel, Wk.sidx, Wk.start, T,
                       reinterpret_cast<double2*>(pos_out), reinterpret_cast<double2*>(u), status, nbr_count,
                       guard_rows, ext_part, reinterpret_cast<unsigned long long*>(solves), Wk.hardq,
                       reinterpret_cast<int32_t*>(Wk.qrec), Wk.qcap, Wk.sctl);
    const long nw = lattice_ext_waves(n);
    const int hb = lattice_wide_blocks(n);
    int hh = 0;  // the hard role's blocks (their extents records follow the main kernel's waves)
    if (CBF_HOCBF_CERT) {
        hh = kSubQ * kHocbfHardPerQ;
        hipLaunchKernelGGL(k_lattice_filter_hocbf_rest, dim3(hh + hb), dim3(64), 0, s, make_kp(p), make_hp(hp), G, W,
                           row_begin, row_end, win_row0, Wk.spos, Wk.svel, Wk.sidx, Wk.start, T,
                           reinterpret_cast<double2*>(pos_out), reinterpret_cast<double2*>(u), status, nbr_count,
                           guard_rows, ext_part ? ext_part + 4l * nw : nullptr,
                           reinterpret_cast<unsigned long long*>(solves), Wk.hardq,
                           reinterpret_cast<int32_t*>(Wk.qrec), Wk.qcap, hh);
    } else {
        hipLaunchKernelGGL(k_lattice_filter_hocbf_wide, dim3(hb), dim3(64), 0, s, make_kp(p), make_hp(hp), G, W,
                           row_begin, row_end, win_row0, Wk.spos, Wk.svel, Wk.sidx, Wk.start, T,
                           reinterpret_cast<double2*>(pos_out), reinterpret_cast<double2*>(u), status, nbr_count,
                           guard_rows, ext_part ? ext_part + 4l * nw : nullptr,
                           reinterpret_cast<unsigned long long*>(solves), Wk.hardq,
                           reinterpret_cast<const int32_t*>(Wk.qrec), Wk.qcap);
    }
    if (extents) launch_extents_finalize((int)(nw + hh) + hb, ext_part, extents, s);
    return (int)hipGetLastError();
}
