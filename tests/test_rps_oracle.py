"""rps-lite restatement (oracle/rps_lite.py): the exact Goldfarb-Idnani
certificate solve is KKT-certified and agrees with the restated cvxopt coneqp; the unicycle maps
keep their documented invariants.  rps itself is absent: parity against it is unpinned."""
import numpy as np
import pytest

from oracle import cvxqp
from oracle import rps_lite as R


def cert_cases(rng, n):
    """Random certificate inputs: spread / clustered / collinear swarms, velocities toward the
    centre (pair rows bind) and at random."""
    out = []
    for t in range(n):
        N = int(rng.integers(1, 17)) if t % 10 else int(rng.integers(17, 33))
        spread = float(rng.choice([0.12, 0.3, 0.6, 1.5]))
        x = rng.uniform(-spread, spread, (2, N))
        if t % 5 == 0 and N > 1:
            x[:, 1] = x[:, 0] + [0.05, 0.0]       # a pair inside the safety radius
        if t % 7 == 0:
            x[1, :] = 0.0                          # collinear swarm
        if t % 2:
            dxi = -x * rng.uniform(0.5, 3.0) + rng.normal(0, 0.05, (2, N))
        else:
            dxi = rng.normal(0, 0.3, (2, N))
        out.append((dxi, x))
    return out


def _lp_min_violation(A, b):
    """min_v max_i (A v - b)_i, clipped at 0 (HiGHS LP): > 0 certifies an empty polyhedron."""
    from scipy.optimize import linprog
    n = A.shape[1]
    c = np.zeros(n + 1)
    c[-1] = 1.0
    r = linprog(c, A_ub=np.hstack([A, -np.ones((A.shape[0], 1))]), b_ub=b, bounds=[(None, None)] * n + [(0, None)],
                method="highs")
    assert r.status == 0
    return r.fun


@pytest.mark.parametrize("seed", [5, 11])
def test_gi_kkt_certificates(seed):
    rng = np.random.default_rng(seed)
    n_active = []
    for dxi, x in cert_cases(rng, 250 if seed == 5 else 400):
        out, info = R.si_barrier_cert(dxi, x, safety_radius=0.12)
        if info["status"] == R.CERT_INFEASIBLE:
            # independent certificate of infeasibility: the best any v can do still violates a row
            assert _lp_min_violation(info["A"], info["b"]) > 1e-9 * max(1.0, float(np.abs(info["b"]).max()))
            assert np.array_equal(out, np.reshape(info["y"], (2, -1), order="F"))
            continue
        assert info["status"] == R.CERT_OPTIMAL
        viol, stat, lmin, comp = R.kkt_residuals(info["y"], info["A"], info["b"], info["x"], info["active"],
                                                 info["lam"])
        sc = max(1.0, float(np.abs(info["b"]).max()))
        assert viol <= 1e-12 * sc and stat <= 1e-12 and comp <= 1e-12 * sc and lmin >= -1e-12
        assert np.array_equal(out, np.reshape(info["x"], (2, -1), order="F"))
        n_active.append(len(info["active"]))
    assert max(n_active) >= 10        # the cases do exercise large active sets


def test_gi_matches_tight_coneqp():
    rng = np.random.default_rng(6)
    for dxi, x in cert_cases(rng, 60):
        _, info = R.si_barrier_cert(dxi, x, safety_radius=0.12)
        n = info["y"].shape[0]
        sol = cvxqp.coneqp(2 * np.eye(n), -2 * info["y"], info["A"], info["b"], maxiters=200, abstol=1e-12,
                           reltol=1e-12, feastol=1e-12)
        assert np.abs(sol["x"] - info["x"]).max() <= 1e-6


def test_gi_infeasible_returns_thresholded_input():
    # two agents on top of each other pushed into one another and boxed in: +-e rows contradict
    y = np.array([0.1, 0.0, -0.1, 0.0])
    A = np.array([[1.0, 0, 0, 0], [-1.0, 0, 0, 0]])
    b = np.array([-1.0, -1.0])                     # x0 <= -1 and x0 >= 1
    res = R.goldfarb_idnani(y, A, b)
    assert res["status"] == R.CERT_INFEASIBLE


def test_threshold_and_rows_follow_rps_order():
    x = np.array([[0.0, 0.3, -0.5], [0.0, 0.1, 0.9]])
    dxi = np.array([[0.3, 0.01, 0.0], [0.4, 0.0, -0.1]])
    y, A, b = R.si_barrier_qp(dxi, x, safety_radius=0.12)
    assert A.shape == (3 + 12, 6)
    assert np.allclose(y[:2], [0.12, 0.16]) and y[2] == 0.01 and y[5] == -0.1   # |(0.3, 0.4)| = 0.5 -> 0.2
    e = x[:, 0] - x[:, 1]
    assert np.array_equal(A[0, :4], np.concatenate([-2 * e, 2 * e]))
    assert b[0] == 100 * np.power((e[0] * e[0] + e[1] * e[1]) - np.power(0.12, 2), 3)
    assert np.array_equal(A[3, :2], [0, 1]) and np.array_equal(A[4, :2], [0, -1])
    assert np.array_equal(A[5, :2], [1, 0]) and np.array_equal(A[6, :2], [-1, 0])


def test_unicycle_maps():
    rng = np.random.default_rng(7)
    poses = np.vstack([rng.uniform(-1, 1, (2, 50)), rng.uniform(-np.pi, np.pi, 50)])
    dxi = rng.normal(0, 0.01, (2, 50))
    dxu = R.si_to_uni_dyn(dxi, poses)
    # inside the angular limit the map is the exact inverse of the projection-point kinematics
    small = np.abs(dxu[1]) < np.pi
    th = poses[2]
    back = np.vstack([np.cos(th) * dxu[0] - 0.05 * np.sin(th) * dxu[1],
                      np.sin(th) * dxu[0] + 0.05 * np.cos(th) * dxu[1]])
    assert np.allclose(back[:, small], dxi[:, small], atol=1e-15)
    v = R.set_velocities(np.array([[0.5, -0.5, 0.1], [10.0, -10.0, 0.0]]))
    assert np.array_equal(v[0], [0.2, -0.2, 0.1]) and np.allclose(np.abs(v[1, :2]), R.MAX_ANGULAR_VELOCITY)
    w = R.wheel_threshold(v)
    dd = np.vstack((1 / (2 * R.WHEEL_RADIUS) * (2 * w[0] - R.BASE_LENGTH * w[1]),
                    1 / (2 * R.WHEEL_RADIUS) * (2 * w[0] + R.BASE_LENGTH * w[1])))
    assert np.all(np.abs(dd) <= R.MAX_WHEEL_VELOCITY * (1 + 1e-12))
    p2 = R.unicycle_step(poses, np.zeros((2, 50)))
    assert np.allclose(p2[:2], poses[:2]) and np.all(np.abs(p2[2]) <= np.pi)


@pytest.mark.slow
def test_cross_and_rescue_shipped_rollout_is_safe_and_bounded():
    from oracle import pyoracle as po
    p = po.Params(15)
    poses, obs = R.cross_and_rescue_initial()
    for _ in range(150):
        poses, obs, rec = R.cross_and_rescue_step(poses, obs, p)
        assert rec["cert_status"] == R.CERT_OPTIMAL
        assert np.all(np.abs(poses[0]) <= 1.6) and np.all(np.abs(poses[1]) <= 1.0)
    # the robots moved toward the goal at (1.5, 0)
    assert poses[0].mean() > -1.15


def test_meet_at_center_shipped_rollout_runs():
    from oracle import pyoracle as po
    p = po.Params(15)
    poses = R.meet_at_center_initial(10)
    ran = 0
    for _ in range(200):
        poses, rec = R.meet_at_center_step(poses, p)
        ran += int((rec["cnt"] > 0).sum())
        assert np.all(np.isfinite(poses)) and np.all(np.abs(poses[2]) <= np.pi)
    assert ran > 0
