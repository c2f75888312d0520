/* Host-side sanitizer driver ("-fsanitize=address on the host C/C++"): exercises the C ABI's
 * host code (cbf_amd/csrc/abi.cpp: cbf_params_init, cbf_abi_version) and the C oracle
 * (oracle/cbf_oracle.c) on random and edge-case inputs under AddressSanitizer and UBSan.
 * Built and run by tests/test_sanitize.py; exits 0 when every check passes. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cbf_amd.h"

typedef struct {
    double max_speed, dmin, k, gamma;
    double f[16];
    double g[8];
    double cull_t;
} orc_params;

void orc_assemble(const orc_params* p, const double r[4], int m, const double* obs, const double u0[2], double* A,
                  double* b);
int orc_filter_one(const orc_params* p, const double r[4], int m, const double* obs, const double u0[2], double u[2],
                   double x[2], int* iters);
void orc_filter_swarm(const orc_params* p, int n, int n_obs, const double* pos, const double* vel, int ego_begin,
                      int ego_end, double* u, int32_t* status, int32_t* cnt, int32_t* nbr_idx, uint8_t* nbr_active,
                      int kmax, uint8_t* box_active, double* xdev, double* viol, double* viol_orig, double* d2min);
void orc_consensus_csr(int n_dst, int self_offset, int n_group, const double* src, const double* anchors,
                       const int32_t* row_ptr, const int32_t* col, int rotate, double rc, double rs, double scale,
                       double* out);
void orc_consensus_lattice(int W, int H, int row_begin, int row_end, const double* pos, double scale, double* out);
void orc_euler(int n, double* pos, const double* vel, double T);
void orc_mc_rollout(const orc_params* p, int n_scen, int n_o, int n_a, int steps, double T, double rc, double rs,
                    double so, double ga, double* pos, int64_t* counters, double* maxviol, double* safety);
int orc_filter_one_hocbf(const orc_params* p, double a_sum, double a_prod, const double r[4], int m, const double* obs,
                         const double u0[2], double u[2], double x[2], int* iters);
void orc_filter_swarm_hocbf(const orc_params* p, double a_sum, double a_prod, int n, int n_obs, const double* pos,
                            const double* vel, int ego_begin, int ego_end, double* u, int32_t* status, int32_t* cnt,
                            double* xdev);

static unsigned long long rng = 88172645463325252ull;
static double urand(double lo, double hi) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return lo + (hi - lo) * (double)(rng >> 11) / 9007199254740992.0;
}

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

static orc_params oparams(const cbf_params* c) {
    orc_params o;
    o.max_speed = c->max_speed;
    o.dmin = c->dmin;
    o.k = c->k;
    o.gamma = c->gamma;
    memcpy(o.f, c->f, sizeof(o.f));
    memcpy(o.g, c->g, sizeof(o.g));
    o.cull_t = c->cull_t;
    return o;
}

int main(void) {
    CHECK(cbf_abi_version() == CBF_ABI_VERSION);
    cbf_params c;
    CHECK(cbf_params_init(&c, 15.0, 0.2, 1.0, NULL, NULL, 0.2) == 0);
    CHECK(c.cull_t < 0.04000000000000001 && sqrt(c.cull_t) >= 0.2 && c.f_is_zero == 1);
    CHECK(cbf_params_init(&c, NAN, 0.2, 1.0, NULL, NULL, 0.2) == CBF_EINVAL);
    CHECK(cbf_params_init(&c, 15.0, 0.2, 1.0, NULL, NULL, -1.0) == CBF_EINVAL);
    CHECK(cbf_params_init(NULL, 15.0, 0.2, 1.0, NULL, NULL, 0.2) == CBF_EINVAL);
    double f16[16], g8[8];
    for (int i = 0; i < 16; ++i) f16[i] = urand(-0.3, 0.3);
    for (int i = 0; i < 8; ++i) g8[i] = urand(-0.3, 0.3);
    CHECK(cbf_params_init(&c, 3.0, 0.3, 2.0, f16, g8, 0.25) == 0 && c.f_is_zero == 0);
    for (int pass = 0; pass < 2; ++pass) {
        CHECK(cbf_params_init(&c, 15.0, 0.2, pass ? 2.0 : 1.0, pass ? f16 : NULL, pass ? g8 : NULL, 0.2) == 0);
        orc_params p = oparams(&c);
        /* single egos: empty and long neighbour lists, assembly rows */
        for (int m = 0; m < 40; m += 7) {
            double r[4], u0[2], u[2], x[2], *obs = malloc(sizeof(double) * 4 * (m ? m : 1));
            double* A = malloc(sizeof(double) * 2 * (m + 8));
            double* b = malloc(sizeof(double) * (m + 8));
            for (int i = 0; i < 4; ++i) r[i] = urand(-1, 1);
            u0[0] = urand(-1, 1), u0[1] = urand(-1, 1);
            for (int i = 0; i < 4 * m; ++i) obs[i] = urand(-1, 1);
            int it;
            const int st = orc_filter_one(&p, r, m, obs, u0, u, x, &it);
            CHECK(st >= 1 && st <= 4 && fabs(u[0]) <= c.max_speed && fabs(u[1]) <= c.max_speed);
            orc_assemble(&p, r, m, obs, u0, A, b);
            const int sh = orc_filter_one_hocbf(&p, 2.0, 1.0, r, m, obs, u0, u, x, &it);
            CHECK(sh >= 1 && sh <= 4);
            free(obs), free(A), free(b);
        }
        /* a swarm with every diagnostic, then one with none; n = 0 is a no-op */
        const int n = 300, n_obs = 30, ne = n - n_obs, kmax = 8;
        double *pos = malloc(sizeof(double) * 2 * n), *vel = malloc(sizeof(double) * 2 * n);
        for (int i = 0; i < 2 * n; ++i) pos[i] = urand(-0.8, 0.8), vel[i] = urand(-0.5, 0.5);
        pos[2 * 40] = pos[2 * 41], pos[2 * 40 + 1] = pos[2 * 41 + 1]; /* coincident agents */
        double *u = malloc(sizeof(double) * 2 * ne), *xd = malloc(sizeof(double) * 2 * ne);
        double *vi = malloc(sizeof(double) * ne), *vo = malloc(sizeof(double) * ne), *d2 = malloc(sizeof(double) * ne);
        int32_t *st = malloc(sizeof(int32_t) * ne), *cnt = malloc(sizeof(int32_t) * ne);
        int32_t* idx = malloc(sizeof(int32_t) * ne * kmax);
        uint8_t *act = malloc((size_t)ne * kmax), *bact = malloc((size_t)ne);
        orc_filter_swarm(&p, n, n_obs, pos, vel, n_obs, n, u, st, cnt, idx, act, kmax, bact, xd, vi, vo, d2);
        for (int k = 0; k < ne; ++k) {
            CHECK((st[k] & 0xFF) <= 4 && cnt[k] >= 0 && cnt[k] < n);
            CHECK(cnt[k] > 0 ? d2[k] < c.cull_t : isinf(d2[k]));
        }
        orc_filter_swarm(&p, n, n_obs, pos, vel, n_obs, n, u, st, cnt, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL);
        orc_filter_swarm(&p, 0, 0, pos, vel, 0, 0, u, st, cnt, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL);
        orc_filter_swarm_hocbf(&p, 2.0, 1.0, n, n_obs, pos, vel, n_obs, n, u, st, cnt, xd);
        orc_euler(n, pos, vel, 1.0 / 30.0);
        /* consensus: CSR with an anchor, and a lattice */
        int32_t rp[4] = {0, 2, 3, 5}, col[5] = {1, 2, 0, 3, 1};
        double src[6] = {0, 0, 1, 0, 0, 1}, anc[2] = {1.5, 0.0}, out[6];
        orc_consensus_csr(3, 0, 3, src, anc, rp, col, 1, cos(0.3), sin(0.3), 0.05, out);
        double* lat = malloc(sizeof(double) * 2 * 12 * 9), * lout = malloc(sizeof(double) * 2 * 12 * 9);
        for (int i = 0; i < 2 * 12 * 9; ++i) lat[i] = urand(0, 2);
        orc_consensus_lattice(12, 9, 0, 9, lat, 0.25, lout);
        orc_consensus_lattice(12, 9, 3, 5, lat, 0.25, lout);
        /* Monte-Carlo rollout with the safety record */
        const int ns = 3, no = 5, na = 4;
        double* mp = malloc(sizeof(double) * 2 * ns * (no + na));
        for (int i = 0; i < 2 * ns * (no + na); ++i) mp[i] = urand(-0.5, 0.5);
        int64_t ctr[12];
        double mv[3], sf[6];
        orc_mc_rollout(&p, ns, no, na, 20, 1.0 / 30.0, cos(-0.6), sin(-0.6), 1.0, 0.5, mp, ctr, mv, sf);
        orc_mc_rollout(&p, ns, no, na, 3, 1.0 / 30.0, cos(-0.6), sin(-0.6), 1.0, 0.5, mp, ctr, mv, NULL);
        for (int s = 0; s < ns; ++s) CHECK(ctr[4 * s] >= ctr[4 * s + 1] && mv[s] >= 0.0);
        free(pos), free(vel), free(u), free(xd), free(vi), free(vo), free(d2), free(st), free(cnt), free(idx);
        free(act), free(bact), free(lat), free(lout), free(mp);
    }
    if (fails) {
        fprintf(stderr, "%d check(s) failed\n", fails);
        return 1;
    }
    printf("sanitize driver ok\n");
    return 0;
}
