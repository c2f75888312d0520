"""Restatement of cvxopt's ``solvers.qp`` -> ``coneqp`` for the QPs of the reference filter.

TEST INFRASTRUCTURE ONLY (the checker: imported by ``tests/`` and bench.py's ``cpu_baseline``
leg, never by ``cbf_amd``).

Why it exists.  The reference solves ``min 1/2|x|^2 s.t. A x <= b`` with
``cvxopt.solvers.qp(Q, p, A, b)`` (/root/reference/cbf.py:64-65,75-81) and the north star asks
for controls within 1e-5 of cvxopt.  cvxopt is a third-party dependency absent from this image
(unpinned in /root/reference/requirements.txt:2; ``import cvxopt`` -> ModuleNotFoundError, an
ordinary error).  Its algorithm is published (L. Vandenberghe, "The CVXOPT linear and quadratic
cone program solvers", 2010, section "Quadratic cone programs"; cvxopt 1.3.x
``coneprog.coneqp``), so this module restates that algorithm for the only cone the reference
uses -- the nonnegative orthant, ``dims = {'l': m, 'q': [], 's': []}``, no equality rows:

* initial point from the W = I KKT system, shifted into the cone by ``1 + max_step``;
* Nesterov-Todd scaling for the orthant (``W = diag(d)``, ``d = sqrt(s/z)``,
  ``lambda = sqrt(s.*z)``);
* Mehrotra predictor-corrector, ``EXPON = 3``, ``STEP = 0.99``, ``sigma = (1 - a + dsdz/gap a^2)^3``;
* the ``chol2`` KKT solver: Cholesky of ``P + G' W^-2 G`` (a failure is ``ArithmeticError``);
* stopping rule ``pres <= feastol and dres <= feastol and (gap <= abstol or relgap <= reltol)``
  with cvxopt's defaults (abstol 1e-7, reltol 1e-6, feastol 1e-7) and the reference's
  ``maxiters = 600`` (cbf.py:76);
* ``ValueError("Rank(A) < p or Rank([P; A; G]) < n")`` only when the KKT factorisation fails at
  iteration 0; a later failure ends the run with status ``'unknown'`` and the current iterate
  ("Terminated (singular KKT matrix)"), as does reaching ``maxiters``.

It is *not* cvxopt: rounding differs (numpy vs cvxopt's BLAS/LAPACK calls), so agreement with the
real binary is within the solver's own tolerances, and parity against cvxopt itself stays
unpinned.  What it pins is the algorithmic claim behind the north star's 1e-5 gate: an
interior-point iterate that meets cvxopt's stopping rule lies within 1e-5 of the exact minimiser
the GPU path computes.  It also shows what the reference returns on an infeasible QP (no
``ValueError`` is raised, so the +1 retry of cbf.py:84-87 never runs; the iterate at
``maxiters`` or at a singular KKT matrix is returned with status ``'unknown'``).
"""
from __future__ import annotations

import math

import numpy as np

EXPON = 3
STEP = 0.99


class _KKT:
    """chol2 factorisation of [P G'; G -W'W] for W = diag(d) (cvxopt kktsolver 'chol2')."""

    def __init__(self, P, G, d):
        K = P + G.T @ (G / (d * d)[:, None])
        n = K.shape[0]
        L = np.zeros_like(K)
        for j in range(n):  # dpotrf: fails on a non-positive or NaN pivot
            a = K[j, j] - L[j, :j] @ L[j, :j]
            if not (a > 0.0) or not math.isfinite(a):
                raise ArithmeticError("potrf")
            L[j, j] = math.sqrt(a)
            for i in range(j + 1, n):
                L[i, j] = (K[i, j] - L[i, :j] @ L[j, :j]) / L[j, j]
        self.L, self.G, self.d = L, G, d

    def solve(self, bx, bz):
        """[P G'; G -W'W] [ux; W^-1 uz] = [bx; bz]  ->  (ux, uz)."""
        L, G, d = self.L, self.G, self.d
        r = bx + G.T @ (bz / (d * d))
        n = len(r)
        y = np.empty(n)
        for i in range(n):
            y[i] = (r[i] - L[i, :i] @ y[:i]) / L[i, i]
        ux = np.empty(n)
        for i in reversed(range(n)):
            ux[i] = (y[i] - L[i + 1:, i] @ ux[i + 1:]) / L[i, i]
        uz = (G @ ux - bz) / d
        return ux, uz


def coneqp(P, q, G, h, maxiters=100, abstol=1e-7, reltol=1e-6, feastol=1e-7):
    """cvxopt.solvers.qp(P, q, G, h) restricted to the orthant.  Returns a dict with keys
    'x', 's', 'z', 'status' ('optimal' | 'unknown'), 'iterations', 'gap', 'pres', 'dres',
    'singular' (terminated on a singular KKT matrix)."""
    P = np.asarray(P, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64).reshape(-1)
    G = np.asarray(G, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64).reshape(-1)
    m = G.shape[0]
    resx0 = max(1.0, float(np.linalg.norm(q)))
    resz0 = max(1.0, float(np.linalg.norm(h)))
    try:
        f = _KKT(P, G, np.ones(m))
    except ArithmeticError:
        raise ValueError("Rank(A) < p or Rank([P; A; G]) < n")
    x, z = f.solve(-q, h)
    s = -z
    nrms, ts = float(np.linalg.norm(s)), float(-s.min())
    if ts >= -1e-8 * max(nrms, 1.0):
        s = s + (1.0 + ts)
    nrmz, tz = float(np.linalg.norm(z)), float(-z.min())
    if tz >= -1e-8 * max(nrmz, 1.0):
        z = z + (1.0 + tz)
    gap = float(s @ z)
    d = lmbda = None

    def result(status, it, singular=False, pres=None, dres=None):
        return {"x": x, "s": s, "z": z, "status": status, "iterations": it, "gap": gap, "pres": pres,
                "dres": dres, "singular": singular}

    for iters in range(maxiters + 1):
        rx = P @ x + q
        f0 = 0.5 * (float(x @ rx) + float(x @ q))
        rx = rx + G.T @ z
        resx = float(np.linalg.norm(rx))
        rz = s + G @ x - h
        resz = float(np.linalg.norm(rz))
        pcost = f0
        dcost = f0 + float(z @ rz) - gap
        if pcost < 0.0:
            relgap = gap / -pcost
        elif dcost > 0.0:
            relgap = gap / dcost
        else:
            relgap = None
        pres, dres = resz / resz0, resx / resx0
        if pres <= feastol and dres <= feastol and (gap <= abstol or (relgap is not None and relgap <= reltol)):
            return result("optimal", iters, pres=pres, dres=dres)
        if iters == maxiters:
            return result("unknown", iters, pres=pres, dres=dres)
        if iters == 0:
            d = np.sqrt(s / z)
            lmbda = np.sqrt(s * z)
        lmbdasq = lmbda * lmbda
        try:
            f3 = _KKT(P, G, d)
        except ArithmeticError:
            if iters == 0:
                raise ValueError("Rank(A) < p or Rank([P; A; G]) < n")
            return result("unknown", iters, singular=True, pres=pres, dres=dres)

        def f4(bx, bz, bs):
            bs = bs / lmbda
            bz = bz - d * bs
            ux, uz = f3.solve(bx, bz)
            return ux, uz, bs - uz

        mu = gap / m
        sigma = eta = 0.0
        ws3 = None
        for i in (0, 1):
            ds = -lmbdasq + sigma * mu
            if i == 1:
                ds = ds - ws3
            dx, dz, ds = f4(-(1.0 - eta) * rx, -(1.0 - eta) * rz, ds)
            dsdz = float(ds @ dz)
            if i == 0:
                ws3 = ds * dz
            ds = ds / lmbda
            dz = dz / lmbda
            t = max(0.0, float(-ds.min()), float(-dz.min()))
            if t == 0.0:
                step = 1.0
            else:
                step = min(1.0, 1.0 / t) if i == 0 else min(1.0, STEP / t)
            if i == 0:
                sigma = min(1.0, max(0.0, 1.0 - step + dsdz / gap * step ** 2)) ** EXPON
                eta = 0.0
        x = x + step * dx
        ds = (1.0 + step * ds) * lmbda
        dz = (1.0 + step * dz) * lmbda
        ssq, zsq = np.sqrt(ds), np.sqrt(dz)
        d = d * ssq / zsq
        lmbda = ssq * zsq
        s = lmbda * d
        z = lmbda / d
        gap = float(lmbda @ lmbda)
    raise AssertionError("unreachable")


def reference_qp(A, b, n_cbf, maxiters=600):
    """cbf.py:64-87 around the restated solver: Q = I, p = 0, the +1 retry of every CBF rhs on
    ValueError.  Returns (solution dict, retries)."""
    A = np.asarray(A, dtype=np.float64)
    b = np.array(b, dtype=np.float64).reshape(-1)
    tries = 0
    while True:
        try:
            return coneqp(np.eye(2), np.zeros(2), A, b, maxiters=maxiters), tries
        except ValueError:
            b[:n_cbf] = b[:n_cbf] + 1.0
            tries += 1


def get_safe_control(A, b, n_cbf, u0, max_speed, maxiters=600):
    """u of cbf.py:89-92 from the restated cvxopt solve (no clip when the caller skips the filter)."""
    sol, _ = reference_qp(A, b, n_cbf, maxiters)
    x = sol["x"]
    u = np.array([x[0] + u0[0], x[1] + u0[1]])
    u[0] = max(min(u[0], max_speed), -max_speed)
    u[1] = max(min(u[1], max_speed), -max_speed)
    return u, sol
