"""Pure-Python CPU restatement of the reference CBF hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: it may be imported by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` and nothing else.  The product path (``cbf_amd``) never imports it
and fails loudly when its HIP library is missing.

Parity pinning: the row assembly, box rows, de-bias and clip below are checked
bit-for-bit against golden vectors captured from the reference's own
``cbf.py`` (see ``tests/golden/make_golden.py``).  The QP minimiser is
checked against an independent brute-force enumerator and KKT certificates;
cvxopt itself is absent from this image, so "within 1e-5 of cvxopt" is
*unpinned* ("Oracle").

Every function cites the reference line(s) it restates.  All arithmetic is
IEEE fp64 in the exact evaluation order the reference's numpy expressions use
(orders were probed against numpy 2.2 / OpenBLAS 0.3.29 and are pinned by the
golden fixtures):

* ``hs_p @ d``             -> ddot: fma chain fma(h3,d3,fma(h2,d2,fma(h1,d1,fma(h0,d0,+0))))
                              (cbf.py:58)
* ``-hs_p @ g``            -> dgemv_n tail: (+0 + fma(h0,g0c,h1*g1c)) + fma(h2,g2c,h3*g3c)
                              (cbf.py:56)
* ``g @ u0`` (gemv)        -> fma(g[r,0], u0x, g[r,1]*u0y)         (cbf.py:59)
* ``np.dot(hs_p, g@u0)``   -> fma chain as hs_p @ d                (cbf.py:59)
* ``f @ d`` (gemv 4x4)     -> dgemv_t: per row (f0 d0 + f2 d2) + (f1 d1 + f3 d3), plain products
                              (cbf.py:55)
* every BLAS result        -> ``+0.0 + r``: BLAS accumulates into a zeroed output, so a
                              result is never -0.0 (only the sign of a zero differs)
The f @ d and -hs_p @ g orders are those of OpenBLAS 0.3.29's x86_64 kernels in this image
(numpy 2.2); the golden fixtures with random f, random g and non-integer k pin them.
* ``np.sum(X[:,j]-X[:,i,None], 1)`` -> sequential from +0.0        (cross_and_rescue.py:118,125)
* ``v @ rotation``         -> fma(v1, R[1,c], v0*R[0,c])           (cross_and_rescue.py:118)
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

GAMMA = 0.5  # cbf.py:16 (hard-coded, not a constructor argument)

# per-agent status codes (low byte); bits 8.. hold the relaxation count
STATUS_IDLE = 0            # no neighbour: filter not called, u = u0 unclipped (cross_and_rescue.py:153)
STATUS_OPTIMAL = 1         # exact minimiser of the QP of cbf.py:62-81
STATUS_RELAXED = 2         # CBF rows relaxed k times by +1 (cbf.py:84-87 rule), then optimal
STATUS_BOX_INFEASIBLE = 3  # the 8 box rows alone are infeasible; x = 0
STATUS_RELAX_CAP = 4       # relaxation cap hit; x = 0

FEAS_TOL = 1e-12   # a.x - b <= FEAS_TOL*max(1,|b|) counts as feasible
ACTIVE_TOL = 1e-12  # a.x >= b - ACTIVE_TOL*max(1,|b|) counts as active
RELAX_CAP = 1 << 16

# cbf.py:66 -- G rows in reference order (rows 1 and 2 are the "mismatched" pair)
BOX_G = ((1.0, 0.0), (0.0, 1.0), (-1.0, 0.0), (0.0, -1.0),
         (1.0, 0.0), (-1.0, 0.0), (0.0, 1.0), (0.0, -1.0))


def fma(a: float, b: float, c: float) -> float:
    """Correctly rounded a*b+c (math.fma is not in Python 3.10)."""
    a = float(a); b = float(b); c = float(c)
    p = a * b
    if c == 0.0 or a == 0.0 or b == 0.0:
        return p + c
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def dot4(h, v):
    """numpy (4,) @ float(4,[1]) as measured (OpenBLAS ddot's scalar tail): a sequential fma
    chain accumulated from +0.0, so the result is never -0.0."""
    return 0.0 + fma(h[3], v[3], fma(h[2], v[2], fma(h[1], v[1], h[0] * v[0])))


def gemv4(f, d):
    """numpy f(4,4) @ d(4,1) as measured (OpenBLAS dgemv_t, 4 lanes then a horizontal add):
    per row (f0 d0 + f2 d2) + (f1 d1 + f3 d3), products rounded, into a zeroed output."""
    return [0.0 + ((f[i, 0] * d[0] + f[i, 2] * d[2]) + (f[i, 1] * d[1] + f[i, 3] * d[3])) for i in range(4)]


def cull_threshold(safety_distance: float) -> float:
    """Smallest t with sqrt(t) >= safety_distance, so that
    ``sqrt(s) < safety_distance  <=>  s < t`` for every double s >= 0
    (cross_and_rescue.py:142-143; for 0.2 this is the double 0.04, *not* 0.2*0.2)."""
    d = float(safety_distance)
    t = d * d
    while t > 0.0 and math.sqrt(np.nextafter(t, 0.0)) >= d:
        t = float(np.nextafter(t, 0.0))
    while math.sqrt(t) < d:
        t = float(np.nextafter(t, math.inf))
    return t


class Params:
    """ControlBarrierFunction(max_speed, dmin=0.2, k=1) state (cbf.py:6-16) plus
    the callers' dynamics f, g (cross_and_rescue.py:31-32) and cull radius (:134)."""

    def __init__(self, max_speed, dmin=0.2, k=1, f=None, g=None, safety_distance=0.2, gamma=GAMMA):
        self.max_speed = float(max_speed)
        self.dmin = float(dmin)
        self.k = float(k)
        self.gamma = float(gamma)
        self.f = np.zeros((4, 4)) if f is None else np.asarray(f, dtype=np.float64).reshape(4, 4)
        self.g = (0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]])) if g is None else \
            np.asarray(g, dtype=np.float64).reshape(4, 2)
        self.safety_distance = float(safety_distance)
        self.cull_t = cull_threshold(safety_distance)


def _hs(p: Params, d0: float, d1: float):
    # cbf.py:47-53 : +1 unless strictly negative (so -0.0 -> +1)
    sx = -1.0 if d0 < 0 else 1.0
    sy = -1.0 if d1 < 0 else 1.0
    return (sx, sy, p.k * sx, p.k * sy), (1 if sx < 0 else 0) | (2 if sy < 0 else 0)


def quadrant_normal(p: Params, q: int):
    """L_g = -hs_p @ g for sign quadrant q (cbf.py:56), numpy's order (OpenBLAS dgemv_n's
    two-row tail: pairs of columns with one fma each, accumulated from +0.0)."""
    sx = -1.0 if (q & 1) else 1.0
    sy = -1.0 if (q & 2) else 1.0
    nh = (-sx, -sy, -(p.k * sx), -(p.k * sy))
    g = p.g
    return tuple(0.0 + ((0.0 + fma(nh[0], g[0, c], nh[1] * g[1, c])) + fma(nh[2], g[2, c], nh[3] * g[3, c]))
                 for c in range(2))


def assemble_row(p: Params, r, o, u0):
    """One barrier row (cbf.py:38-59). Returns (a0, a1, b, quadrant)."""
    d = [float(r[i]) - float(o[i]) for i in range(4)]                 # cbf.py:39
    hs, q = _hs(p, d[0], d[1])                                          # cbf.py:47-53
    H = dot4(hs, d)                                                     # hs_p @ d
    fd = gemv4(p.f, d)                                                  # f @ d
    L_f = dot4(hs, fd)                                                  # cbf.py:55
    a0, a1 = quadrant_normal(p, q)                                       # cbf.py:56
    g = p.g
    gu = [0.0 + fma(g[i, 0], u0[0], g[i, 1] * u0[1]) for i in range(4)]  # g @ u0
    c = dot4(hs, gu)
    b = (p.gamma * (H - p.dmin) + L_f) + c                               # cbf.py:58-59
    return a0, a1, b, q


def box_rhs(p: Params, r, u0):
    """S_saturated (cbf.py:67-70), reference row order."""
    ms = p.max_speed
    u0x, u0y = float(u0[0]), float(u0[1])
    rvx, rvy = float(r[2]), float(r[3])
    return [ms - u0x, ms + u0x, ms - u0y, ms + u0y,
            (ms - rvx) - u0x, (ms + rvx) + u0x, (ms - rvy) - u0y, (ms + rvy) + u0y]


def assemble(p: Params, r, obs, u0):
    """A = vstack(L_gs, G), b = vstack(rhs, S) exactly as handed to cvxopt (cbf.py:72-80)."""
    rows = [assemble_row(p, r, o, u0) for o in obs]
    A = [(a0, a1) for a0, a1, _, _ in rows] + list(BOX_G)
    b = [bb for _, _, bb, _ in rows] + box_rhs(p, r, u0)
    return np.array(A, dtype=np.float64).reshape(-1, 2), np.array(b, dtype=np.float64)


# --------------------------------------------------------------------------------------
# exact 2-variable QP:  min 1/2|x|^2  s.t.  a_h . x <= b_h   (cbf.py:62-81, Q=I, p=0)
# --------------------------------------------------------------------------------------
def _viol_ok(a0, a1, b, tb, x0, x1):
    return (a0 * x0 + a1 * x1) - b <= tb


def solve_halfplanes(planes):
    """Exact min-norm point of a list of half-planes a.x <= b (<= 8, fixed order
    [box+x, box+y, box-x, box-y, cbf q0..q3 present]).  Incremental (Seidel) method:
    keep the optimum of the prefix; when plane h is violated the new optimum lies on its
    line, found by clamping t=0 (the origin's projection) to the interval cut out by the
    earlier planes.  Feasibility tolerance FEAS_TOL*max(1,|b|) in b-units.
    Returns (fail_index, x0, x1): fail_index = -1 when feasible, else the plane index at which
    the prefix became infeasible (< 4 means the box rows alone are infeasible)."""
    n = len(planes)
    tb = [FEAS_TOL * _py_max(1.0, abs(b)) for (_, _, b) in planes]
    x0 = 0.0
    x1 = 0.0
    for h in range(n):
        a0, a1, b = planes[h]
        if _viol_ok(a0, a1, b, tb[h], x0, x1):
            continue
        n2 = a0 * a0 + a1 * a1
        if not (n2 > 0):
            return h, 0.0, 0.0
        t = b / n2
        p0 = t * a0
        p1 = t * a1
        d0 = -a1
        d1 = a0
        # interval of s on the line: bounds r/ad compared by cross-multiplication,
        # only the binding one divided out
        hi = lo = None              # (r, ad) of the binding upper / lower bound
        for j in range(h):
            c0, c1, e = planes[j]
            ad = c0 * d0 + c1 * d1
            r = e - (c0 * p0 + c1 * p1)
            if ad > 0:
                if hi is None or r * hi[1] < hi[0] * ad:
                    hi = (r, ad)
            elif ad < 0:
                if lo is None or r * lo[1] > lo[0] * ad:
                    lo = (r, ad)
        s = 0.0
        s_hi = False
        if hi is not None and hi[0] < 0:
            s = hi[0] / hi[1]
            s_hi = True
        if lo is not None and ((hi[0] * lo[1] > lo[0] * hi[1]) if s_hi else (lo[0] < 0)):
            s = lo[0] / lo[1]
        x0 = p0 + s * d0
        x1 = p1 + s * d1
        for j in range(h + 1):
            c0, c1, e = planes[j]
            if not _viol_ok(c0, c1, e, tb[j], x0, x1):
                return h, 0.0, 0.0
    return -1, x0, x1


def _box_planes(S):
    return [(1.0, 0.0, min(S[0], S[4])), (0.0, 1.0, min(S[1], S[6])),
            (-1.0, 0.0, min(S[2], S[5])), (0.0, -1.0, min(S[3], S[7]))]


def _py_min(a, b):
    return b if b < a else a


def _py_max(a, b):
    return b if b > a else a


def clip(p: Params, x0, x1, u0):
    """cbf.py:89-91 -- u = x + u0, then Python max(min(u, ms), -ms) per component."""
    ms = p.max_speed
    u = [x0 + float(u0[0]), x1 + float(u0[1])]
    return [_py_max(_py_min(v, ms), -ms) for v in u]


def filter_one(p: Params, r, obs, u0):
    """get_safe_control (cbf.py:18-92) for one ego with its culled neighbour list.
    Returns dict(u, x, status, iters, rows=(A,b) of the final (possibly relaxed) QP)."""
    u0 = [float(u0[0]), float(u0[1])]
    bq = [None] * 4
    for o in obs:
        _, _, b, q = assemble_row(p, r, o, u0)
        bq[q] = b if bq[q] is None else _py_min(bq[q], b)
    S = box_rhs(p, r, u0)
    box = _box_planes(S)
    normals = [quadrant_normal(p, q) for q in range(4)]

    def planes_for(bqv):
        return box + [(normals[q][0], normals[q][1], bqv[q]) for q in range(4) if bqv[q] is not None]

    fail, x0, x1 = solve_halfplanes(planes_for(bq))
    status, iters = STATUS_OPTIMAL, 0
    if fail >= 0:
        if fail < 4:                                   # box rows alone infeasible
            status, x0, x1 = STATUS_BOX_INFEASIBLE, 0.0, 0.0
        else:
            while True:
                bq = [None if v is None else v + 1.0 for v in bq]   # cbf.py:85-87
                iters += 1
                fail, x0, x1 = solve_halfplanes(planes_for(bq))
                if fail < 0:
                    status = STATUS_RELAXED
                    break
                if iters >= RELAX_CAP:
                    status, x0, x1 = STATUS_RELAX_CAP, 0.0, 0.0
                    break
    u = clip(p, x0, x1, u0)
    return dict(u=u, x=[x0, x1], status=status, iters=iters)


def relaxed_b(b: float, iters: int) -> float:
    for _ in range(iters):
        b = b + 1.0
    return b


def diagnose(p: Params, r, obs, u0, x, iters):
    """Active set and violation of the final QP at x (SURVEY 8d correctness gates)."""
    A, b = assemble(p, r, obs, u0)
    m = len(obs)
    active, viol = [], 0.0
    for i in range(A.shape[0]):
        bi = relaxed_b(float(b[i]), iters) if i < m else float(b[i])
        lhs = A[i, 0] * x[0] + A[i, 1] * x[1]
        active.append(bool(lhs >= bi - ACTIVE_TOL * max(1.0, abs(bi))))
        viol = max(viol, lhs - bi)
    return active, max(viol, 0.0)


# --------------------------------------------------------------------------------------
# callers: cull, nominal control, Euler  (cross_and_rescue.py / meet_at_center.py)
# --------------------------------------------------------------------------------------
def cull_one(p: Params, pos, n_obs, ego):
    """Neighbour indices of ego (cross_and_rescue.py:141-150): every obstacle with
    dist < 0.2 (index order), then every agent with 0 < dist < 0.2 (index order)."""
    r0, r1 = float(pos[ego][0]), float(pos[ego][1])
    out = []
    for j in range(len(pos)):
        e0 = float(pos[j][0]) - r0
        e1 = float(pos[j][1]) - r1
        s = (0 + e0 * e0) + e1 * e1       # builtin sum over (o-r)**2
        if s < p.cull_t and (j < n_obs or s > 0):
            out.append(j)
    return out


def filter_swarm(p: Params, pos, vel, n_obs, ego_begin, ego_end):
    """The per-agent loop of cross_and_rescue.py:135-160 (Jacobi: every ego sees the
    nominal states packed before the loop, :133).  Ego state = [pos, vel] with
    vel = its nominal control u0 (:133,155)."""
    pos = np.asarray(pos, dtype=np.float64)
    vel = np.asarray(vel, dtype=np.float64)
    n = ego_end - ego_begin
    u = np.zeros((n, 2)); status = np.zeros(n, np.int32); cnt = np.zeros(n, np.int32)
    nbrs = []
    for e in range(ego_begin, ego_end):
        nb = cull_one(p, pos, n_obs, e)
        nbrs.append(nb)
        k = e - ego_begin
        cnt[k] = len(nb)
        if not nb:
            u[k] = vel[e]                 # not filtered, not clipped (cross_and_rescue.py:153)
            status[k] = STATUS_IDLE
            continue
        r = [pos[e, 0], pos[e, 1], vel[e, 0], vel[e, 1]]
        obs = [[pos[j, 0], pos[j, 1], vel[j, 0], vel[j, 1]] for j in nb]
        res = filter_one(p, r, obs, vel[e])
        u[k] = res["u"]
        status[k] = res["status"] | (min(res["iters"], (1 << 23) - 1) << 8)
    return u, status, cnt, nbrs


def consensus_csr(src, row_ptr, col, self_idx, n_group, anchors=None, scale=1.0, rot=None):
    """Nominal control by graph Laplacian (cross_and_rescue.py:108-125,
    meet_at_center.py:86-103):  v_i = (sum_j (x_j - x_i)) [@ R(theta)] * scale.
    col >= n_group refers to anchors[col - n_group] (the goal column, cross_and_rescue.py:102)."""
    out = np.zeros((len(self_idx), 2))
    for k, i in enumerate(self_idx):
        xi = src[i]
        acc = [0.0, 0.0]
        for jj in range(row_ptr[k], row_ptr[k + 1]):
            j = col[jj]
            xj = src[j] if j < n_group else anchors[j - n_group]
            acc[0] = acc[0] + (float(xj[0]) - float(xi[0]))
            acc[1] = acc[1] + (float(xj[1]) - float(xi[1]))
        if rot is not None:
            c, s = rot
            v = [fma(acc[1], -s, acc[0] * c), fma(acc[1], c, acc[0] * s)]
        else:
            v = acc
        out[k] = [v[0] * scale, v[1] * scale]
    return out


def lattice_neighbors(i, W, H):
    """4-neighbour lattice Laplacian row, ascending index (np.where order)."""
    r, c = divmod(i, W)
    out = []
    if r > 0: out.append(i - W)
    if c > 0: out.append(i - 1)
    if c < W - 1: out.append(i + 1)
    if r < H - 1: out.append(i + W)
    return out


def euler(pos, vel, T):
    """p <- p + T*v (cross_and_rescue.py:173)."""
    return np.asarray(pos) + T * np.asarray(vel)


_M1, _M2, _GOLD = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB), np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def random_nominal(pos, g0, amp, seed):
    """The synthetic random-walk nominal control of the lattice builds (include/cbf_amd.h
    CBF_NOMINAL_RANDOM; no reference counterpart -- cfg4 names a synthetic swarm, not its nominal
    controller): for agent g0 + i at pos[i], h = splitmix64 finalisers chained over (seed + gold
    (g + 1), bits(x), bits(y)); u0 = amp (2 U - 1) per component, U = (h >> 11) 2^-53 for x and
    the same of mix(h + gold) for y.  Integer arithmetic mod 2^64, then one rounding (amp * v)."""
    pos = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 2)
    g = np.arange(pos.shape[0], dtype=np.uint64) + np.uint64(g0 + 1)
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(seed) + _GOLD * g)
        h = _mix64(h ^ pos[:, 0].copy().view(np.uint64))
        h = _mix64(h ^ pos[:, 1].copy().view(np.uint64))
        h2 = _mix64(h + _GOLD)
    v0 = 2.0 * ((h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53) - 1.0
    v1 = 2.0 * ((h2 >> np.uint64(11)).astype(np.float64) * 2.0 ** -53) - 1.0
    return np.stack([amp * v0, amp * v1], axis=1)


# --------------------------------------------------------------------------------------
# Euclidean HOCBF barrier mode (BASELINE.json north star (2)).
# The reference has no such mode, so there is no reference oracle: this restatement
# defines the arithmetic (Python == C oracle == device, bit for bit) and the QP minimiser
# is certified by the brute-force KKT check of tests/golden/qp_bruteforce.py.
#
# Double integrator per agent: p' = v, v' = u.  For ego i and neighbour j (constant
# velocity, u_j = 0 -- the decentralised convention of cbf.py, which reads neighbour states
# only):  h = |p_i - p_j|^2 - Ds^2,  h' = 2 dp.dv,  h'' = 2|dv|^2 + 2 dp.u,
# psi1 = h' + a1 h,  psi2 = psi1' + a2 psi1 = h'' + (a1 + a2) h' + a1 a2 h >= 0, i.e.
#     (-2 dp) . u  <=  2|dv|^2 + (a1 + a2) h' + a1 a2 h                    (Ds = dmin)
# and with x = u - u0 (cbf.py's decision variable):  (-2 dp) . x <= rhs - (-2 dp) . u0.
# Box rows, +1 relaxation, de-bias and clip are the reference's (cbf.py:62-92) unchanged;
# every barrier row is its own half-plane (no per-quadrant merge), in neighbour order.
# --------------------------------------------------------------------------------------
class HocbfParams:
    def __init__(self, alpha1=1.0, alpha2=1.0):
        self.alpha1 = float(alpha1)
        self.alpha2 = float(alpha2)
        self.a_sum = self.alpha1 + self.alpha2
        self.a_prod = self.alpha1 * self.alpha2


def hocbf_row(p: Params, hp: HocbfParams, r, o, u0):
    """(a0, a1, b) of one Euclidean HOCBF row; evaluation order fixed (no fma)."""
    dx = float(r[0]) - float(o[0])
    dy = float(r[1]) - float(o[1])
    dvx = float(r[2]) - float(o[2])
    dvy = float(r[3]) - float(o[3])
    h = (dx * dx + dy * dy) - p.dmin * p.dmin
    hd = 2.0 * (dx * dvx + dy * dvy)
    vv = dvx * dvx + dvy * dvy
    rhs = (2.0 * vv + hp.a_sum * hd) + hp.a_prod * h
    a0 = -2.0 * dx
    a1 = -2.0 * dy
    return a0, a1, rhs - (a0 * float(u0[0]) + a1 * float(u0[1]))


def filter_one_hocbf(p: Params, hp: HocbfParams, r, obs, u0):
    """get_safe_control with Euclidean HOCBF rows: box planes first (merged as in the
    reference mode), then one plane per neighbour in order; +1 relaxation of every barrier
    row while infeasible (cbf.py:84-87 rule)."""
    u0 = [float(u0[0]), float(u0[1])]
    rows = [hocbf_row(p, hp, r, o, u0) for o in obs]
    box = _box_planes(box_rhs(p, r, u0))
    fail, x0, x1 = solve_halfplanes(box + rows)
    status, iters = STATUS_OPTIMAL, 0
    if fail >= 0:
        if fail < 4:
            status, x0, x1 = STATUS_BOX_INFEASIBLE, 0.0, 0.0
        else:
            while True:
                rows = [(a0, a1, b + 1.0) for (a0, a1, b) in rows]
                iters += 1
                fail, x0, x1 = solve_halfplanes(box + rows)
                if fail < 0:
                    status = STATUS_RELAXED
                    break
                if iters >= RELAX_CAP:
                    status, x0, x1 = STATUS_RELAX_CAP, 0.0, 0.0
                    break
    return dict(u=clip(p, x0, x1, u0), x=[x0, x1], status=status, iters=iters, rows=box + rows)


def filter_swarm_hocbf(p: Params, hp: HocbfParams, pos, vel, n_obs, ego_begin, ego_end):
    """filter_swarm (cross_and_rescue.py:135-160 loop) with Euclidean HOCBF rows; the ego
    state is (pos, vel) with u0 = vel as in the reference mode."""
    pos = np.asarray(pos, dtype=np.float64)
    vel = np.asarray(vel, dtype=np.float64)
    n = ego_end - ego_begin
    u = np.zeros((n, 2)); status = np.zeros(n, np.int32); cnt = np.zeros(n, np.int32)
    for e in range(ego_begin, ego_end):
        nb = cull_one(p, pos, n_obs, e)
        k = e - ego_begin
        cnt[k] = len(nb)
        if not nb:
            u[k] = vel[e]
            continue
        r = [pos[e, 0], pos[e, 1], vel[e, 0], vel[e, 1]]
        obs = [[pos[j, 0], pos[j, 1], vel[j, 0], vel[j, 1]] for j in nb]
        res = filter_one_hocbf(p, hp, r, obs, vel[e])
        u[k] = res["u"]
        status[k] = res["status"] | (min(res["iters"], (1 << 23) - 1) << 8)
    return u, status, cnt
