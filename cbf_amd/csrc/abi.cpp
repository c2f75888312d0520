// abi.cpp -- host-side parameter setup of the C ABI (ControlBarrierFunction.__init__, cbf.py:6-16).
#include <math.h>
#include <string.h>

#include "cbf_amd.h"

// Smallest t with sqrt(t) >= d, so that sqrt(s) < d <=> s < t (cross_and_rescue.py:142-143).
static double cull_threshold(double d) {
    double t = d * d;
    while (t > 0.0 && sqrt(nextafter(t, 0.0)) >= d) t = nextafter(t, 0.0);
    while (sqrt(t) < d) t = nextafter(t, INFINITY);
    return t;
}

extern "C" int cbf_params_init(cbf_params* p, double max_speed, double dmin, double k, const double* f16,
                               const double* g8, double safety_distance) {
    if (!p || !(safety_distance >= 0) || !isfinite(max_speed) || !isfinite(dmin) || !isfinite(k)) return CBF_EINVAL;
    memset(p, 0, sizeof(*p));
    p->max_speed = max_speed;
    p->dmin = dmin;
    p->k = k;
    p->gamma = 0.5;  // cbf.py:16
    int fz = 1;
    for (int i = 0; i < 16; ++i) {
        p->f[i] = f16 ? f16[i] : 0.0;
        if (p->f[i] != 0.0) fz = 0;
    }
    static const double g_callers[8] = {0.1, 0.0, 0.0, 0.1, 0.0, 0.0, 0.0, 0.0};  // 0.1*[[1,0],[0,1],[0,0],[0,0]]
    for (int i = 0; i < 8; ++i) p->g[i] = g8 ? g8[i] : g_callers[i];
    p->f_is_zero = fz;
    p->cull_t = cull_threshold(safety_distance);
    p->relax_cap = 1 << 16;
    p->solve_inline_max = -1;  // the library's threshold (swarm.hip kSolveInlineDefault)
    // L_g = -hs_p @ g per sign quadrant (cbf.py:56) in numpy's order: OpenBLAS dgemv_n's two-row
    // tail, one fma per pair of columns, accumulated into a zeroed output (oracle/pyoracle.py)
    for (int q = 0; q < 4; ++q) {
        const double sx = (q & 1) ? -1.0 : 1.0, sy = (q & 2) ? -1.0 : 1.0;
        const double nh[4] = {-sx, -sy, -(k * sx), -(k * sy)};
        for (int c = 0; c < 2; ++c) {
            const double t01 = fma(nh[0], p->g[0 * 2 + c], nh[1] * p->g[1 * 2 + c]);
            const double t23 = fma(nh[2], p->g[2 * 2 + c], nh[3] * p->g[3 * 2 + c]);
            p->nrm[q][c] = 0.0 + ((0.0 + t01) + t23);
        }
    }
    return 0;
}

extern "C" int cbf_abi_version(void) { return CBF_ABI_VERSION; }
