"""Euclidean HOCBF barrier mode, CPU side: the Python and C restatements agree bit for bit, and
the QP minimiser is certified by the independent brute-force enumerator + KKT check (there is no
reference oracle for this mode -- parity is to this restatement)."""
import os
import sys

import numpy as np
import pytest

from oracle import coracle, pyoracle as po

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import qp_bruteforce as bf  # noqa: E402


def _cases(rng, n):
    for _ in range(n):
        m = int(rng.integers(0, 12))
        r = np.concatenate([rng.uniform(-1, 1, 2), rng.normal(0, 0.5, 2)])
        obs = np.concatenate([r[:2] + rng.uniform(-0.3, 0.3, (m, 2)), rng.normal(0, 0.5, (m, 2))], axis=1)
        if m > 2 and rng.random() < 0.2:
            obs[1] = obs[0]                       # duplicate row
        if m > 3 and rng.random() < 0.1:
            obs[2, :2] = r[:2]                    # coincident position: zero normal
        u0 = rng.normal(0, 0.5, 2)
        hp = po.HocbfParams(*rng.choice([0.5, 1.0, 2.0, 3.0], 2))
        yield po.Params(float(rng.choice([1.0, 15.0])), dmin=float(rng.choice([0.1, 0.2]))), hp, r, obs, u0


def test_python_equals_c():
    rng = np.random.default_rng(21)
    for p, hp, r, obs, u0 in _cases(rng, 400):
        a = po.filter_one_hocbf(p, hp, r, obs, u0)
        b = coracle.filter_one_hocbf(p, hp, r, obs, u0)
        assert a["status"] == b["status"] and a["iters"] == b["iters"]
        assert np.array_equal(np.array(a["u"]), b["u"]) and np.array_equal(np.array(a["x"]), b["x"])


def test_minimiser_kkt_certified():
    rng = np.random.default_rng(22)
    n_relaxed = 0
    for p, hp, r, obs, u0 in _cases(rng, 300):
        res = po.filter_one_hocbf(p, hp, r, obs, u0)
        if res["status"] not in (po.STATUS_OPTIMAL, po.STATUS_RELAXED):
            continue
        n_relaxed += res["status"] == po.STATUS_RELAXED
        # the final (relaxed, if so) planes; row order is irrelevant to the unique minimiser
        A = np.array([[a0, a1] for a0, a1, _ in res["rows"]])
        b = np.array([bb for _, _, bb in res["rows"]])
        x_bf = bf.solve(A, b)
        assert x_bf is not None
        assert np.abs(np.array(res["x"]) - x_bf).max() <= 1e-9
        assert bf.kkt_residual(A, b, np.array(res["x"])) <= 1e-9
        if res["iters"] > 0:  # one relaxation fewer is infeasible (the count is minimal)
            b1 = np.array([po.hocbf_row(p, hp, r, o, u0)[2] for o in obs])
            for _ in range(res["iters"] - 1):
                b1 = b1 + 1.0
            assert bf.solve(A, np.concatenate([b[:4], b1])) is None
    assert n_relaxed > 0


def test_head_on_neighbour_brakes():
    """One neighbour straight ahead, closing at 0.04 m/s: the filtered acceleration pushes away."""
    p, hp = po.Params(15, dmin=0.2), po.HocbfParams(1.0, 1.0)
    r = [0.0, 0.0, 0.04, 0.0]  # inside the safe set psi1 >= 0, psi2 < 0 at u = 0
    res = po.filter_one_hocbf(p, hp, r, [[0.25, 0.0, 0.0, 0.0]], [0.0, 0.0])
    assert res["status"] == po.STATUS_OPTIMAL
    assert res["u"][0] < 0 and abs(res["u"][1]) < 1e-15
    # the psi2 >= 0 row holds with equality at the optimum
    a0, a1, b = res["rows"][4]
    assert abs((a0 * res["x"][0] + a1 * res["x"][1]) - b) <= 1e-12


@pytest.mark.parametrize("n,n_obs", [(60, 10), (400, 0)])
def test_swarm_python_equals_c(n, n_obs):
    rng = np.random.default_rng(n)
    p, hp = po.Params(15), po.HocbfParams(1.0, 2.0)
    pos = rng.uniform(-1.0, 1.0, (n, 2))
    vel = rng.normal(0, 0.3, (n, 2))
    u, st, cnt = po.filter_swarm_hocbf(p, hp, pos, vel, n_obs, n_obs, n)
    c = coracle.filter_swarm_hocbf(p, hp, pos, vel, n_obs)
    assert np.array_equal(u, c["u"]) and np.array_equal(st, c["status"]) and np.array_equal(cnt, c["cnt"])
