/*
 * cbf_oracle.c -- C restatement of the reference CBF hot path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the *checker*.  Never linked by the product
 * library (cbf_amd/libcbf_amd.so).
 *
 * It restates, operation for operation, oracle/pyoracle.py (which is pinned
 * bit-for-bit to golden vectors captured from the reference's cbf.py); the C
 * and Python restatements are cross-checked bit-exactly in tests/.
 * Reference lines restated:
 *   row assembly            cbf.py:38-59
 *   box rows                cbf.py:63-70
 *   QP (exact, 2 vars)      cbf.py:62-87   (retry rule cbf.py:84-87 on infeasibility)
 *   de-bias + clip          cbf.py:89-91
 *   cull                    cross_and_rescue.py:141-150, meet_at_center.py:124-133
 *   consensus / pursuit     cross_and_rescue.py:108-125, meet_at_center.py:86-103
 *   Euler                   cross_and_rescue.py:173
 *   Euclidean HOCBF mode    (no reference: restates oracle/pyoracle.py hocbf_row / filter_one_hocbf)
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double max_speed, dmin, k, gamma;
    double f[16]; /* row-major 4x4 */
    double g[8];  /* row-major 4x2 */
    double cull_t;
} orc_params;

enum { ST_IDLE = 0, ST_OPTIMAL = 1, ST_RELAXED = 2, ST_BOX_INFEASIBLE = 3, ST_RELAX_CAP = 4 };
#define FEAS_TOL 1e-12
#define ACTIVE_TOL 1e-12
#define RELAX_CAP (1 << 16)

/* numpy's orders (OpenBLAS 0.3.29 x86_64 kernels, pinned by tests/golden; pyoracle.py header):
 * every BLAS result is accumulated into a zeroed output, hence the "0.0 +" (never -0.0) */
static double dot4(const double h[4], const double v[4]) { /* ddot */
    return 0.0 + fma(h[3], v[3], fma(h[2], v[2], fma(h[1], v[1], h[0] * v[0])));
}

/* f(4x4) @ d (dgemv_t: 4 lanes, then a horizontal add) */
static void gemv4(const double f[16], const double d[4], double fd[4]) {
    for (int i = 0; i < 4; ++i)
        fd[i] = 0.0 + ((f[i * 4 + 0] * d[0] + f[i * 4 + 2] * d[2]) + (f[i * 4 + 1] * d[1] + f[i * 4 + 3] * d[3]));
}

/* -hs_p @ g (dgemv_n's two-row tail) */
static void quadrant_normal(const orc_params* p, int q, double a[2]) {
    double sx = (q & 1) ? -1.0 : 1.0, sy = (q & 2) ? -1.0 : 1.0;
    double nh[4] = {-sx, -sy, -(p->k * sx), -(p->k * sy)};
    for (int c = 0; c < 2; ++c)
        a[c] = 0.0 + ((0.0 + fma(nh[0], p->g[0 * 2 + c], nh[1] * p->g[1 * 2 + c])) +
                      fma(nh[2], p->g[2 * 2 + c], nh[3] * p->g[3 * 2 + c]));
}

/* cbf.py:38-59 */
static double row_b(const orc_params* p, const double r[4], const double o[4], const double u0[2], int* quad) {
    double d[4];
    for (int i = 0; i < 4; ++i) d[i] = r[i] - o[i];
    double sx = (d[0] < 0) ? -1.0 : 1.0, sy = (d[1] < 0) ? -1.0 : 1.0;
    double hs[4] = {sx, sy, p->k * sx, p->k * sy};
    double H = dot4(hs, d);
    double fd[4];
    gemv4(p->f, d, fd);
    double L_f = dot4(hs, fd);
    double gu[4];
    for (int i = 0; i < 4; ++i) gu[i] = 0.0 + fma(p->g[i * 2 + 0], u0[0], p->g[i * 2 + 1] * u0[1]);
    double c = dot4(hs, gu);
    *quad = (sx < 0 ? 1 : 0) | (sy < 0 ? 2 : 0);
    return (p->gamma * (H - p->dmin) + L_f) + c;
}

/* cbf.py:67-70 */
static void box_rhs(const orc_params* p, const double r[4], const double u0[2], double S[8]) {
    double ms = p->max_speed;
    S[0] = ms - u0[0];
    S[1] = ms + u0[0];
    S[2] = ms - u0[1];
    S[3] = ms + u0[1];
    S[4] = (ms - r[2]) - u0[0];
    S[5] = (ms + r[2]) + u0[0];
    S[6] = (ms - r[3]) - u0[1];
    S[7] = (ms + r[3]) + u0[1];
}

static const double BOX_G[8][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}, {1, 0}, {-1, 0}, {0, 1}, {0, -1}};

void orc_assemble(const orc_params* p, const double r[4], int m, const double* obs, const double u0[2], double* A,
                  double* b) {
    for (int i = 0; i < m; ++i) {
        int q;
        b[i] = row_b(p, r, obs + 4 * i, u0, &q);
        quadrant_normal(p, q, A + 2 * i);
    }
    double S[8];
    box_rhs(p, r, u0, S);
    for (int i = 0; i < 8; ++i) {
        A[2 * (m + i)] = BOX_G[i][0];
        A[2 * (m + i) + 1] = BOX_G[i][1];
        b[m + i] = S[i];
    }
}

static double py_min(double a, double b) { return (b < a) ? b : a; }
static double py_max(double a, double b) { return (b > a) ? b : a; }

typedef struct {
    int n;
    double a0[8], a1[8], b[8];
} planes_t;

/* Incremental (Seidel) exact min-norm solve over the planes in order; returns -1 when
 * feasible (x set) or the index of the plane at which the prefix became infeasible. */
static int solve_planes_n(int n, const double* A0, const double* A1, const double* B, double* x0o, double* x1o) {
    double x0 = 0.0, x1 = 0.0;
    for (int h = 0; h < n; ++h) {
        double a0 = A0[h], a1 = A1[h], b = B[h];
        if ((a0 * x0 + a1 * x1) - b <= FEAS_TOL * py_max(1.0, fabs(b))) continue;
        double n2 = a0 * a0 + a1 * a1;
        if (!(n2 > 0)) return h;
        double t = b / n2;
        double p0 = t * a0, p1 = t * a1;
        double d0 = -a1, d1 = a0;
        /* interval of t on the line: bounds r/ad compared by cross-multiplication, only the
         * binding one divided out */
        double rh = 0.0, ah = 0.0, rl = 0.0, al = 0.0;
        int has_hi = 0, has_lo = 0;
        for (int j = 0; j < h; ++j) {
            double c0 = A0[j], c1 = A1[j], e = B[j];
            double ad = c0 * d0 + c1 * d1;
            double r = e - (c0 * p0 + c1 * p1);
            if (ad > 0) {
                if (!has_hi || r * ah < rh * ad) {
                    rh = r;
                    ah = ad;
                }
                has_hi = 1;
            } else if (ad < 0) {
                if (!has_lo || r * al > rl * ad) {
                    rl = r;
                    al = ad;
                }
                has_lo = 1;
            }
        }
        double s = 0.0;
        int s_hi = 0;
        if (has_hi && rh < 0) {
            s = rh / ah;
            s_hi = 1;
        }
        if (has_lo && (s_hi ? (rh * al > rl * ah) : (rl < 0))) s = rl / al;
        x0 = p0 + s * d0;
        x1 = p1 + s * d1;
        for (int j = 0; j <= h; ++j)
            if (!((A0[j] * x0 + A1[j] * x1) - B[j] <= FEAS_TOL * py_max(1.0, fabs(B[j])))) return h;
    }
    *x0o = x0;
    *x1o = x1;
    return -1;
}

static int solve_planes(const planes_t* P, double* x0o, double* x1o) {
    return solve_planes_n(P->n, P->a0, P->a1, P->b, x0o, x1o);
}

static void box_planes(const double S[8], planes_t* P) {
    P->n = 4;
    P->a0[0] = 1.0;  P->a1[0] = 0.0;  P->b[0] = py_min(S[0], S[4]);
    P->a0[1] = 0.0;  P->a1[1] = 1.0;  P->b[1] = py_min(S[1], S[6]);
    P->a0[2] = -1.0; P->a1[2] = 0.0;  P->b[2] = py_min(S[2], S[5]);
    P->a0[3] = 0.0;  P->a1[3] = -1.0; P->b[3] = py_min(S[3], S[7]);
}

/* the grouped QP for one ego: returns status, x, iters; bq/present are the per-quadrant min rows */
static int solve_ego(const orc_params* p, const double r[4], const double u0[2], const double bq_in[4],
                     const int present[4], double x[2], int* iters_out, double* viol_out) {
    double S[8];
    box_rhs(p, r, u0, S);
    planes_t P, B;
    box_planes(S, &B);
    double nrm[4][2];
    for (int q = 0; q < 4; ++q) quadrant_normal(p, q, nrm[q]);
    double bq[4] = {bq_in[0], bq_in[1], bq_in[2], bq_in[3]};
    int iters = 0, status = ST_OPTIMAL;
    for (;;) {
        P = B;
        for (int q = 0; q < 4; ++q)
            if (present[q]) {
                P.a0[P.n] = nrm[q][0];
                P.a1[P.n] = nrm[q][1];
                P.b[P.n] = bq[q];
                P.n++;
            }
        int fail = solve_planes(&P, &x[0], &x[1]);
        if (fail < 0) break;
        if (fail < 4) { /* box rows alone infeasible */
            status = ST_BOX_INFEASIBLE;
            x[0] = x[1] = 0.0;
            break;
        }
        if (iters >= RELAX_CAP) {
            status = ST_RELAX_CAP;
            x[0] = x[1] = 0.0;
            break;
        }
        for (int q = 0; q < 4; ++q) bq[q] = bq[q] + 1.0; /* cbf.py:85-87 */
        iters++;
        status = ST_RELAXED;
    }
    if (viol_out) {
        double v = 0.0;
        for (int h = 0; h < P.n; ++h) {
            double lhs = P.a0[h] * x[0] + P.a1[h] * x[1];
            double d = lhs - P.b[h];
            if (d > v) v = d;
        }
        *viol_out = v;
    }
    *iters_out = iters;
    return status;
}

static void clip(const orc_params* p, const double x[2], const double u0[2], double u[2]) {
    double ms = p->max_speed;
    for (int c = 0; c < 2; ++c) u[c] = py_max(py_min(x[c] + u0[c], ms), -ms);
}

/* get_safe_control (cbf.py:18-92) for an explicit neighbour list */
int orc_filter_one(const orc_params* p, const double r[4], int m, const double* obs, const double u0[2], double u[2],
                   double x[2], int* iters) {
    double bq[4] = {0, 0, 0, 0};
    int present[4] = {0, 0, 0, 0};
    for (int i = 0; i < m; ++i) {
        int q;
        double b = row_b(p, r, obs + 4 * i, u0, &q);
        bq[q] = present[q] ? py_min(bq[q], b) : b;
        present[q] = 1;
    }
    int st = solve_ego(p, r, u0, bq, present, x, iters, 0);
    clip(p, x, u0, u);
    return st;
}

/* max(0, a.x - b) over the ego's ORIGINAL rows (merged box rows, per-quadrant barrier minima before
 * any relaxation): the violation of the barrier the reference asked for (a reported statistic;
 * same evaluation order as cbf_device.hpp:orig_violation). */
static double orig_violation(const orc_params* p, const double r[4], const double u0[2], const double bq[4],
                             const int present[4], const double x[2]) {
    double S[8];
    box_rhs(p, r, u0, S);
    const double bb[4] = {py_min(S[0], S[4]), py_min(S[1], S[6]), py_min(S[2], S[5]), py_min(S[3], S[7])};
    const double ab[4] = {x[0], x[1], -x[0], -x[1]};
    double v = 0.0;
    for (int h = 0; h < 4; ++h) v = py_max(v, ab[h] - bb[h]);
    for (int q = 0; q < 4; ++q)
        if (present[q]) {
            double nq[2];
            quadrant_normal(p, q, nq);
            v = py_max(v, (nq[0] * x[0] + nq[1] * x[1]) - bq[q]);
        }
    return v;
}

static double relaxed(double b, int iters) {
    for (int i = 0; i < iters; ++i) b = b + 1.0;
    return b;
}

/*
 * The per-agent loop of cross_and_rescue.py:135-160 over a swarm (Jacobi: all egos see the
 * packed nominal states, :133).  Entities [0,n_obs) are obstacles (no dist>0 test), [n_obs,n)
 * agents.  Ego e's state is (pos[e], vel[e]) and its nominal control is vel[e].
 * Optional diagnostics (any pointer may be NULL): neighbour indices (ascending), per-neighbour
 * active flags, box-row active bits, x (deviation), max violation.
 */
void orc_filter_swarm(const orc_params* p, int n, int n_obs, const double* pos, const double* vel, int ego_begin,
                      int ego_end, double* u, int32_t* status, int32_t* cnt, int32_t* nbr_idx, uint8_t* nbr_active,
                      int kmax, uint8_t* box_active, double* xdev, double* viol, double* viol_orig, double* d2min) {
    for (int e = ego_begin; e < ego_end; ++e) {
        int k = e - ego_begin;
        double r[4] = {pos[2 * e], pos[2 * e + 1], vel[2 * e], vel[2 * e + 1]};
        double u0[2] = {vel[2 * e], vel[2 * e + 1]};
        double bq[4] = {0, 0, 0, 0};
        int present[4] = {0, 0, 0, 0};
        int m = 0;
        double dm = INFINITY;
        for (int j = 0; j < n; ++j) {
            double e0 = pos[2 * j] - r[0], e1 = pos[2 * j + 1] - r[1];
            double s = (0.0 + e0 * e0) + e1 * e1;
            if (!(s < p->cull_t && (j < n_obs || s > 0))) continue;
            dm = py_min(dm, s);
            double o[4] = {pos[2 * j], pos[2 * j + 1], vel[2 * j], vel[2 * j + 1]};
            int q;
            double b = row_b(p, r, o, u0, &q);
            bq[q] = present[q] ? py_min(bq[q], b) : b;
            present[q] = 1;
            if (nbr_idx && m < kmax) nbr_idx[(size_t)k * kmax + m] = j;
            m++;
        }
        cnt[k] = m;
        if (d2min) d2min[k] = dm;
        if (nbr_idx)
            for (int t = m; t < kmax; ++t) nbr_idx[(size_t)k * kmax + t] = -1;
        if (m == 0) {
            u[2 * k] = u0[0];
            u[2 * k + 1] = u0[1];
            status[k] = ST_IDLE;
            if (xdev) xdev[2 * k] = xdev[2 * k + 1] = 0.0;
            if (viol) viol[k] = 0.0;
            if (viol_orig) viol_orig[k] = 0.0;
            if (box_active) box_active[k] = 0;
            if (nbr_active)
                for (int t = 0; t < kmax; ++t) nbr_active[(size_t)k * kmax + t] = 0;
            continue;
        }
        double x[2];
        int iters;
        double v;
        int st = solve_ego(p, r, u0, bq, present, x, &iters, &v);
        double uu[2];
        clip(p, x, u0, uu);
        u[2 * k] = uu[0];
        u[2 * k + 1] = uu[1];
        status[k] = st | ((iters < (1 << 23) ? iters : (1 << 23) - 1) << 8);
        if (xdev) {
            xdev[2 * k] = x[0];
            xdev[2 * k + 1] = x[1];
        }
        if (viol) viol[k] = v;
        if (viol_orig) viol_orig[k] = iters > 0 ? orig_violation(p, r, u0, bq, present, x) : v;
        if (box_active) {
            double S[8];
            box_rhs(p, r, u0, S);
            uint8_t bits = 0;
            for (int i = 0; i < 8; ++i) {
                double lhs = BOX_G[i][0] * x[0] + BOX_G[i][1] * x[1];
                if (lhs >= S[i] - ACTIVE_TOL * py_max(1.0, fabs(S[i]))) bits |= (uint8_t)(1u << i);
            }
            box_active[k] = bits;
        }
        if (nbr_active && nbr_idx) {
            for (int t = 0; t < kmax; ++t) {
                uint8_t act = 0;
                int j = nbr_idx[(size_t)k * kmax + t];
                if (j >= 0) {
                    double o[4] = {pos[2 * j], pos[2 * j + 1], vel[2 * j], vel[2 * j + 1]};
                    int q;
                    double b = relaxed(row_b(p, r, o, u0, &q), iters);
                    double a[2];
                    quadrant_normal(p, q, a);
                    double lhs = a[0] * x[0] + a[1] * x[1];
                    act = lhs >= b - ACTIVE_TOL * py_max(1.0, fabs(b));
                }
                nbr_active[(size_t)k * kmax + t] = act;
            }
        }
    }
}

/* cross_and_rescue.py:108-125 / meet_at_center.py:86-103 over a CSR Laplacian.
 * out[k] for k in [0,n_dst): self = src[self_offset+k]; col >= n_group -> anchors[col-n_group]. */
void orc_consensus_csr(int n_dst, int self_offset, int n_group, const double* src, const double* anchors,
                       const int32_t* row_ptr, const int32_t* col, int rotate, double rc, double rs, double scale,
                       double* out) {
    for (int k = 0; k < n_dst; ++k) {
        int i = self_offset + k;
        double a0 = 0.0, a1 = 0.0;
        for (int t = row_ptr[k]; t < row_ptr[k + 1]; ++t) {
            int j = col[t];
            const double* xj = (j < n_group) ? src + 2 * j : anchors + 2 * (j - n_group);
            a0 = a0 + (xj[0] - src[2 * i]);
            a1 = a1 + (xj[1] - src[2 * i + 1]);
        }
        double v0 = a0, v1 = a1;
        if (rotate) {
            v0 = fma(a1, -rs, a0 * rc);
            v1 = fma(a1, rc, a0 * rs);
        }
        out[2 * k] = v0 * scale;
        out[2 * k + 1] = v1 * scale;
    }
}

/* 4-neighbour lattice Laplacian (rows [row_begin,row_end) of a W x H lattice), ascending index order */
void orc_consensus_lattice(int W, int H, int row_begin, int row_end, const double* pos, double scale, double* out) {
    for (int r = row_begin; r < row_end; ++r)
        for (int c = 0; c < W; ++c) {
            long i = (long)r * W + c;
            long nb[4];
            int m = 0;
            if (r > 0) nb[m++] = i - W;
            if (c > 0) nb[m++] = i - 1;
            if (c < W - 1) nb[m++] = i + 1;
            if (r < H - 1) nb[m++] = i + W;
            double a0 = 0.0, a1 = 0.0;
            for (int t = 0; t < m; ++t) {
                a0 = a0 + (pos[2 * nb[t]] - pos[2 * i]);
                a1 = a1 + (pos[2 * nb[t] + 1] - pos[2 * i + 1]);
            }
            long k = i - (long)row_begin * W;
            out[2 * k] = a0 * scale;
            out[2 * k + 1] = a1 * scale;
        }
}

/* cross_and_rescue.py:173 */
void orc_euler(int n, double* pos, const double* vel, double T) {
    for (int i = 0; i < 2 * n; ++i) pos[i] = pos[i] + T * vel[i];
}

/*
 * Batched Monte-Carlo rendezvous (SURVEY cfg5; generalises meet_at_center.py:76-153):
 * per scenario, n_o pursuit obstacles (ring Laplacian i -> i+1, rotation (rc,rs), scale so)
 * followed by n_a free agents (complete-graph consensus, gain ga); only agents are filtered.
 * pos: [n_scen][n_o+n_a][2], updated in place over `steps` Euler steps of length T.
 * counters: [n_scen][4] int64 = {filter calls, relaxed, box-infeasible, relax-cap}; maxviol [n_scen] = max
 * row violation over OPTIMAL solves; safety [n_scen][2] (nullable) = {max violation of the original rows
 * over RELAXED solves, min neighbour distance^2 of an agent}.
 */
void orc_mc_rollout(const orc_params* p, int n_scen, int n_o, int n_a, int steps, double T, double rc, double rs,
                    double so, double ga, double* pos, int64_t* counters, double* maxviol, double* safety) {
    int n = n_o + n_a;
    double vel[2 * 512];
    double u[2 * 256];
    int32_t st[256], cnt[256];
    double viol[256], vorig[256], d2[256];
    int32_t ring_ptr[2] = {0, 1};
    for (int s = 0; s < n_scen; ++s) {
        double* P = pos + (size_t)s * n * 2;
        int64_t* C = counters + (size_t)s * 4;
        C[0] = C[1] = C[2] = C[3] = 0;
        double mv = 0.0, mvo = 0.0, dmin = INFINITY;
        for (int t = 0; t < steps; ++t) {
            for (int i = 0; i < n_o; ++i) {
                int32_t col = (i + 1) % n_o;
                orc_consensus_csr(1, i, n_o, P, 0, ring_ptr, &col, 1, rc, rs, so, vel + 2 * i);
            }
            for (int i = 0; i < n_a; ++i) {
                int32_t cols[512];
                int m = 0;
                for (int j = 0; j < n_a; ++j)
                    if (j != i) cols[m++] = j;
                int32_t rp[2] = {0, m};
                orc_consensus_csr(1, i, n_a, P + 2 * n_o, 0, rp, cols, 0, 1.0, 0.0, ga, vel + 2 * (n_o + i));
            }
            orc_filter_swarm(p, n, n_o, P, vel, n_o, n, u, st, cnt, 0, 0, 0, 0, 0, viol, vorig, d2);
            for (int i = 0; i < n_a; ++i) {
                dmin = py_min(dmin, d2[i]);
                if (cnt[i] == 0) continue;
                C[0]++;
                int code = st[i] & 0xff;
                if (code == ST_RELAXED) C[1]++;
                if (code == ST_BOX_INFEASIBLE) C[2]++;
                if (code == ST_RELAX_CAP) C[3]++;
                if (code == ST_OPTIMAL) mv = viol[i] > mv ? viol[i] : mv;
                if (code == ST_RELAXED) mvo = vorig[i] > mvo ? vorig[i] : mvo;
                vel[2 * (n_o + i)] = u[2 * i];
                vel[2 * (n_o + i) + 1] = u[2 * i + 1];
            }
            orc_euler(n, P, vel, T);
        }
        maxviol[s] = mv;
        if (safety) {
            safety[2 * s] = mvo;
            safety[2 * s + 1] = dmin;
        }
    }
}

/* ---- Euclidean HOCBF mode (oracle/pyoracle.py: hocbf_row, filter_one_hocbf) ---- */
static void hocbf_row(const orc_params* p, double a_sum, double a_prod, const double r[4], const double o[4],
                      const double u0[2], double* a0, double* a1, double* b) {
    double dx = r[0] - o[0], dy = r[1] - o[1], dvx = r[2] - o[2], dvy = r[3] - o[3];
    double h = (dx * dx + dy * dy) - p->dmin * p->dmin;
    double hd = 2.0 * (dx * dvx + dy * dvy);
    double vv = dvx * dvx + dvy * dvy;
    double rhs = (2.0 * vv + a_sum * hd) + a_prod * h;
    *a0 = -2.0 * dx;
    *a1 = -2.0 * dy;
    *b = rhs - (*a0 * u0[0] + *a1 * u0[1]);
}

/* planes: 4 merged box planes then one per neighbour (scratch arrays of m + 4) */
static int solve_hocbf(const orc_params* p, const double r[4], const double u0[2], int m, double* A0, double* A1,
                       double* B, double x[2], int* iters_out) {
    double S[8];
    box_rhs(p, r, u0, S);
    planes_t bx;
    box_planes(S, &bx);
    for (int i = 0; i < 4; ++i) {
        A0[i] = bx.a0[i];
        A1[i] = bx.a1[i];
        B[i] = bx.b[i];
    }
    int iters = 0, status = ST_OPTIMAL;
    for (;;) {
        int fail = solve_planes_n(m + 4, A0, A1, B, &x[0], &x[1]);
        if (fail < 0) break;
        if (fail < 4) {
            status = ST_BOX_INFEASIBLE;
            x[0] = x[1] = 0.0;
            break;
        }
        if (iters >= RELAX_CAP) {
            status = ST_RELAX_CAP;
            x[0] = x[1] = 0.0;
            break;
        }
        for (int i = 4; i < m + 4; ++i) B[i] = B[i] + 1.0; /* cbf.py:85-87 */
        iters++;
        status = ST_RELAXED;
    }
    *iters_out = iters;
    return status;
}

int orc_filter_one_hocbf(const orc_params* p, double a_sum, double a_prod, const double r[4], int m, const double* obs,
                         const double u0[2], double u[2], double x[2], int* iters) {
    double* A0 = malloc(sizeof(double) * (m + 4));
    double* A1 = malloc(sizeof(double) * (m + 4));
    double* B = malloc(sizeof(double) * (m + 4));
    for (int i = 0; i < m; ++i) hocbf_row(p, a_sum, a_prod, r, obs + 4 * i, u0, &A0[4 + i], &A1[4 + i], &B[4 + i]);
    int st = solve_hocbf(p, r, u0, m, A0, A1, B, x, iters);
    clip(p, x, u0, u);
    free(A0);
    free(A1);
    free(B);
    return st;
}

/* orc_filter_swarm's loop (cull in index order, Jacobi) with Euclidean HOCBF rows */
void orc_filter_swarm_hocbf(const orc_params* p, double a_sum, double a_prod, int n, int n_obs, const double* pos,
                            const double* vel, int ego_begin, int ego_end, double* u, int32_t* status, int32_t* cnt,
                            double* xdev) {
    double* A0 = malloc(sizeof(double) * (n + 4));
    double* A1 = malloc(sizeof(double) * (n + 4));
    double* B = malloc(sizeof(double) * (n + 4));
    for (int e = ego_begin; e < ego_end; ++e) {
        int k = e - ego_begin;
        double r[4] = {pos[2 * e], pos[2 * e + 1], vel[2 * e], vel[2 * e + 1]};
        double u0[2] = {vel[2 * e], vel[2 * e + 1]};
        int m = 0;
        for (int j = 0; j < n; ++j) {
            double e0 = pos[2 * j] - r[0], e1 = pos[2 * j + 1] - r[1];
            double s = (0.0 + e0 * e0) + e1 * e1;
            if (!(s < p->cull_t && (j < n_obs || s > 0))) continue;
            double o[4] = {pos[2 * j], pos[2 * j + 1], vel[2 * j], vel[2 * j + 1]};
            hocbf_row(p, a_sum, a_prod, r, o, u0, &A0[4 + m], &A1[4 + m], &B[4 + m]);
            m++;
        }
        cnt[k] = m;
        double x[2] = {0.0, 0.0};
        if (m == 0) {
            u[2 * k] = u0[0];
            u[2 * k + 1] = u0[1];
            status[k] = ST_IDLE;
        } else {
            int iters;
            int st = solve_hocbf(p, r, u0, m, A0, A1, B, x, &iters);
            double uu[2];
            clip(p, x, u0, uu);
            u[2 * k] = uu[0];
            u[2 * k + 1] = uu[1];
            status[k] = st | ((iters < (1 << 23) ? iters : (1 << 23) - 1) << 8);
        }
        if (xdev) {
            xdev[2 * k] = x[0];
            xdev[2 * k + 1] = x[1];
        }
    }
    free(A0);
    free(A1);
    free(B);
}
