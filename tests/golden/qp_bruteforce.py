"""Independent brute-force solver + KKT certificate for the 2-variable QP
``min 1/2 |x|^2  s.t.  A x <= b`` handed to cvxopt at reference cbf.py:81.

TEST INFRASTRUCTURE ONLY.  Deliberately a *different* formulation from the
oracle's grouped solver: it works on the original m+8 rows (no per-quadrant
merge, no phase ordering) and enumerates every row and every row pair.
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy.optimize import nnls

TOL = 1e-11


def solve(A, b):
    A = np.asarray(A, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(1.0, np.abs(b))

    def feas(x):
        return bool(np.all(A @ x - b <= TOL * scale))

    cands = [np.zeros(2)]
    for i in range(len(b)):
        n2 = A[i] @ A[i]
        if n2 > 0:
            cands.append(A[i] * (b[i] / n2))
    for i, j in itertools.combinations(range(len(b)), 2):
        M = np.array([A[i], A[j]])
        if abs(np.linalg.det(M)) < 1e-300:
            continue
        cands.append(np.linalg.solve(M, np.array([b[i], b[j]])))
    best = None
    for x in cands:
        if feas(x) and (best is None or x @ x < best @ best - 1e-15):
            best = x
    return best  # None when infeasible


def kkt_residual(A, b, x, act_tol=1e-9):
    """Max KKT residual of x: primal violation, and |x + A_act^T lam| with lam >= 0 (NNLS)."""
    A = np.asarray(A, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    r = A @ x - b
    prim = float(max(0.0, r.max()))
    act = np.where(r >= -act_tol * np.maximum(1.0, np.abs(b)))[0]
    if len(act) == 0:
        return max(prim, float(np.abs(x).max()))
    lam, res = nnls(A[act].T, -x)
    return max(prim, float(res))
