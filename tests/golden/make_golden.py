"""Capture golden vectors from the reference's own ``cbf.py``.

Runs ONLY in the build container (``/root/reference`` does not exist on the GPU
box); its outputs (``tests/golden/*.npz``) are committed data fixtures.

How: ``cvxopt`` is absent from this image (ordinary ``ModuleNotFoundError``, no
permission denial -- SURVEY.md 8c).  The reference module is loaded from
``/root/reference/cbf.py`` with a *recording* stand-in for the two cvxopt
entry points it touches (``cvxopt.matrix`` as a column-major container and
``cvxopt.solvers.qp``).  The stand-in performs no arithmetic on the problem
data: every number in the captured ``A``/``b`` is computed by the reference's
own numpy code (cbf.py:38-80), and the reference's own de-bias/clip
(cbf.py:89-91) produces ``u`` from the minimiser the stand-in returns.  That
minimiser comes from the independent brute-force enumerator in
``qp_bruteforce.py`` and is KKT-certified here; cvxopt's own interior-point
iterate is therefore *not* pinned (parity vs cvxopt: unpinned).

The caller-side pieces (scenario geometry cross_and_rescue.py:36-57 /
meet_at_center.py:31-48, consensus :108-125 / :86-103, cull :141-150 / :124-133)
live in module-level scripts that need the absent ``rps`` simulator, so they
are restated here expression-for-expression and recorded alongside.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import qp_bruteforce  # noqa: E402

REF = "/root/reference/cbf.py"


# ----------------------------------------------------------------------------------
# recording stand-in for the cvxopt entry points used at cbf.py:64-81
# ----------------------------------------------------------------------------------
class _Mat:
    def __init__(self, arr):
        a = np.array(arr, dtype=np.float64)
        if a.ndim == 1:
            a = a.reshape(-1, 1)
        self.a = a

    def __getitem__(self, i):           # cvxopt indexes column-major
        return self.a.reshape(-1, order="F")[i]

    @property
    def size(self):
        return self.a.shape


def _matrix(x):
    if isinstance(x, _Mat):
        return _Mat(x.a)
    if isinstance(x, list):             # a list of block-columns, each a list stacked vertically
        cols = [np.vstack([blk.a if isinstance(blk, _Mat) else np.array(blk, dtype=np.float64)
                           for blk in col]) for col in x]
        return _Mat(np.hstack(cols))
    return _Mat(x)


class _Recorder:
    calls = []

    @staticmethod
    def qp(P, q, G, h):
        A = G.a.copy()
        b = h.a.reshape(-1).copy()
        x = qp_bruteforce.solve(A, b)
        iters = 0
        if x is None:
            # Infeasible: cvxopt's iterate is undefined (status unchecked at cbf.py:82).  The
            # framework's *defined* output applies the reference's own retry rule (cbf.py:84-87:
            # every CBF row += 1) until feasible; restated here independently of the oracle.
            m = len(b) - 8
            if qp_bruteforce.solve(A[m:], b[m:]) is None:
                iters, x = -1, np.zeros(2)          # box rows alone infeasible: x = 0
            else:
                bb = b.copy()
                while x is None:
                    bb[:m] = bb[:m] + 1.0
                    iters += 1
                    x = qp_bruteforce.solve(A, bb)
        _Recorder.calls.append((A, b, x, iters))
        return {"x": _Mat(x.reshape(2, 1)), "status": "optimal" if iters == 0 else "unknown"}


def load_reference_cbf():
    shim = types.ModuleType("cvxopt")
    shim.matrix = _matrix
    shim.solvers = types.SimpleNamespace(options={}, qp=_Recorder.qp)
    sys.modules["cvxopt"] = shim
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_cbf", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


FX = 0.1 * np.array([[0, 0, 0, 0], [0, 0, 0, 0], [0, 0, 0, 0], [0, 0, 0, 0]])  # cross_and_rescue.py:31
GX = 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]])                          # cross_and_rescue.py:32


def call(ctrl, r, obs, f, g, u0):
    _Recorder.calls.clear()
    u = ctrl.get_safe_control(np.array(r, dtype=np.float64), np.array(obs, dtype=np.float64), f, g,
                              np.array(u0, dtype=np.float64))
    assert len(_Recorder.calls) == 1
    A, b, x, iters = _Recorder.calls[0]
    return A, b, x, np.asarray(u, dtype=np.float64).reshape(2), iters


# ----------------------------------------------------------------------------------
# filter cases: random + adversarial
# ----------------------------------------------------------------------------------
def filter_cases(mod, rng):
    cases = []  # (r, obs, u0, max_speed, dmin, k, g, tag, f)

    def add(r, obs, u0, ms=15, dmin=0.2, k=1, g=GX, tag=0, f=FX):
        cases.append((np.array(r, float), np.array(obs, float).reshape(-1, 4), np.array(u0, float), ms, dmin, k,
                      np.array(g, float), tag, np.array(f, float)))

    # tag 0: caller-shaped random cases (robot "velocity" slot = u0, cross_and_rescue.py:133)
    for _ in range(1500):
        m = int(rng.integers(1, 13))
        p = rng.uniform(-1.5, 1.5, 2)
        u0 = rng.normal(0, 0.5, 2) * (10 ** rng.uniform(-2, 0.5))
        r = [p[0], p[1], u0[0], u0[1]]
        obs = []
        for _ in range(m):
            ang = rng.uniform(0, 2 * np.pi)
            rad = rng.uniform(0.0, 0.2)
            v = rng.normal(0, 0.5, 2) * (10 ** rng.uniform(-2, 0.5))
            obs.append([p[0] + rad * np.cos(ang), p[1] + rad * np.sin(ang), v[0], v[1]])
        add(r, obs, u0)
    # tag 1: generic robot velocity slot != u0, other speeds / dmin / k
    for _ in range(300):
        m = int(rng.integers(1, 9))
        r = list(rng.uniform(-1, 1, 2)) + list(rng.normal(0, 2, 2))
        u0 = rng.normal(0, 2, 2)
        obs = [list(np.array(r[:2]) + rng.normal(0, 0.1, 2)) + list(rng.normal(0, 2, 2)) for _ in range(m)]
        add(r, obs, u0, ms=float(rng.choice([15, 2.0, 0.5])), dmin=float(rng.choice([0.2, 0.1, 0.35])),
            k=int(rng.choice([1, 2, 3])), tag=1)
    # tag 2: general constant g (pins the -hs@g / g@u0 evaluation orders)
    for _ in range(200):
        m = int(rng.integers(1, 7))
        r = list(rng.uniform(-1, 1, 2)) + list(rng.normal(0, 0.5, 2))
        u0 = rng.normal(0, 0.5, 2)
        obs = [list(np.array(r[:2]) + rng.normal(0, 0.1, 2)) + list(rng.normal(0, 0.5, 2)) for _ in range(m)]
        add(r, obs, u0, g=rng.normal(0, 0.3, (4, 2)), tag=2)
    # tag 3: adversarial -- signed zeros in d, ties in b, coincident obstacles, sandwiches (infeasible)
    for sx in (0.0, -0.0):
        for sy in (0.0, -0.0):
            r = [sx, sy, 0.1, -0.2]
            add(r, [[0.0, 0.0, 0.0, 0.0], [0.0, 0.05, 0.1, 0.0], [-0.0, -0.05, 0.0, 0.1]], [0.1, -0.2], tag=3)
    for _ in range(60):
        p = rng.uniform(-1, 1, 2)
        u0 = rng.normal(0, 0.3, 2)
        o = [p[0] + 0.05, p[1] + 0.03, 0.1, 0.1]
        add([p[0], p[1], u0[0], u0[1]], [o, o, list(o)], u0, tag=3)                      # exact ties
        add([p[0], p[1], u0[0], u0[1]], [[p[0] + 0.02, p[1] + 0.02, 0, 0],
                                          [p[0] - 0.02, p[1] - 0.02, 0, 0]], u0, tag=3)  # sandwich
        add([p[0], p[1], u0[0], u0[1]], [[p[0], p[1], 0.0, 0.0]], u0, tag=3)             # coincident
    # tag 4: large nominal controls -> box rows bind / clip engages / box infeasible
    for _ in range(60):
        r = list(rng.uniform(-1, 1, 2)) + list(rng.normal(0, 12, 2))
        u0 = rng.normal(0, 12, 2)
        obs = [list(np.array(r[:2]) + rng.normal(0, 0.1, 2)) + list(rng.normal(0, 3, 2)) for _ in range(3)]
        add(r, obs, u0, tag=4)
    # the worked example probed in SURVEY 8c: r=(0,0,.3,-.2), two neighbours
    add([0.0, 0.0, 0.3, -0.2], [[0.1, 0.05, 0.0, 0.0], [-0.05, 0.1, 0.2, 0.1]], [0.3, -0.2], tag=5)
    # round 5: the constructor's and get_safe_control's other inputs at non-default values
    # (cbf.py:6 max_speed / dmin / k, cbf.py:55-59 f and g).  Own generator, so the cases above and
    # the rollouts / consensus vectors after them keep their draws.
    r5 = np.random.default_rng(20261018)
    # tag 6: random dynamics f (4x4, L_f = hs_p @ (f @ d), cbf.py:55), callers' g
    for _ in range(250):
        m = int(r5.integers(1, 9))
        r = list(r5.uniform(-1, 1, 2)) + list(r5.normal(0, 0.5, 2))
        u0 = r5.normal(0, 0.5, 2)
        obs = [list(np.array(r[:2]) + r5.normal(0, 0.1, 2)) + list(r5.normal(0, 0.5, 2)) for _ in range(m)]
        f = r5.normal(0, 1, (4, 4)) * (10 ** r5.uniform(-2, 0.5, (4, 4)))
        add(r, obs, u0, ms=float(r5.choice([15, 2.0])), dmin=float(r5.choice([0.2, 0.35])), f=f, tag=6)
    # tag 7: non-integer k (hs_p a float array, cbf.py:47-53), callers' f and g
    for _ in range(200):
        m = int(r5.integers(1, 9))
        r = list(r5.uniform(-1, 1, 2)) + list(r5.normal(0, 0.5, 2))
        u0 = r5.normal(0, 0.5, 2)
        obs = [list(np.array(r[:2]) + r5.normal(0, 0.1, 2)) + list(r5.normal(0, 0.5, 2)) for _ in range(m)]
        add(r, obs, u0, k=float(r5.choice([0.5, 1.5, 0.7, 2.5])), dmin=float(r5.choice([0.2, 0.1])), tag=7)
    # tag 8: everything at once -- random f and g, k in {0.5, 1.5, 2, 2.5}, other max_speed / dmin
    # (the FilterParams the fused-path GPU tests run), plus signed-zero offsets
    for i in range(300):
        m = int(r5.integers(1, 11))
        r = list(r5.uniform(-1, 1, 2)) + list(r5.normal(0, 0.5, 2))
        u0 = r5.normal(0, 0.5, 2)
        obs = [list(np.array(r[:2]) + r5.normal(0, 0.1, 2)) + list(r5.normal(0, 0.5, 2)) for _ in range(m)]
        if i % 10 == 0:
            obs[0][0] = r[0]          # dx = +0.0
            if m > 1:
                obs[1][1] = r[1]      # dy = +0.0
        f = r5.normal(0, 0.5, (4, 4))
        g = r5.normal(0, 0.3, (4, 2))
        add(r, obs, u0, ms=float(r5.choice([15, 2.0, 0.5])), dmin=float(r5.choice([0.2, 0.35])),
            k=float(r5.choice([0.5, 1.5, 2.0, 2.5])), g=g, f=f, tag=8)

    R, OBS_OFF, OBS, U0, MS, DMIN, KK, G, TAG, FF = [], [0], [], [], [], [], [], [], [], []
    A_OFF, A, B, X, U, IT = [0], [], [], [], [], []
    kkt_max = 0.0
    for (r, obs, u0, ms, dmin, k, g, tag, f) in cases:
        # k as the caller passes it: an int (hs_p an int64 array, cbf.py:47) when integral
        ctrl = mod.ControlBarrierFunction(ms, dmin=dmin, k=int(k) if float(k).is_integer() else k)
        Ai, bi, xi, ui, it = call(ctrl, r, obs, f, g, u0)
        FF.append(f)
        if it == 0:
            kkt_max = max(kkt_max, qp_bruteforce.kkt_residual(Ai, bi, xi))
        IT.append(it)
        R.append(r); OBS.append(obs); OBS_OFF.append(OBS_OFF[-1] + len(obs)); U0.append(u0)
        MS.append(ms); DMIN.append(dmin); KK.append(k); G.append(g); TAG.append(tag)
        A.append(Ai); B.append(bi); A_OFF.append(A_OFF[-1] + len(bi)); X.append(xi); U.append(ui)
    print(f"filter cases: {len(cases)}, infeasible: {int((np.array(IT) != 0).sum())}, "
          f"max KKT residual {kkt_max:.2e}")
    assert kkt_max < 1e-9
    return dict(r=np.array(R), obs=np.vstack(OBS), obs_off=np.array(OBS_OFF), u0=np.array(U0),
                max_speed=np.array(MS, float), dmin=np.array(DMIN), k=np.array(KK, float), g=np.array(G),
                f=np.array(FF),
                tag=np.array(TAG), A=np.vstack(A), b=np.concatenate(B), ab_off=np.array(A_OFF),
                x=np.array(X), u=np.array(U), relax_iters=np.array(IT))


# ----------------------------------------------------------------------------------
# caller restatements (rps absent): topology, consensus, cull -- expression for expression
# ----------------------------------------------------------------------------------
def topological_neighbors(L, agent):
    """rps.utilities.graph.topological_neighbors [upstream, unverified]: off-diagonal nonzeros."""
    row = np.array(L[agent, :])
    row[agent] = 0
    return np.where(row != 0)[0]


def completeGL(n):
    """rps.utilities.graph.completeGL [upstream, unverified]: n*I - 1 1^T."""
    return n * np.eye(n) - np.ones((n, n))


def cull(robot_state, obstacle_states, agent_states, safety_distance=0.2):
    """cross_and_rescue.py:137-150 verbatim expressions; returns indices (obstacles, then agents)."""
    idx = []
    for j, obstacle_state in enumerate(obstacle_states):
        distance = np.sqrt(sum((obstacle_state[:2] - robot_state[:2]) ** 2))
        if distance < safety_distance:
            idx.append(j)
    for j, agent_state in enumerate(agent_states):
        distance = np.sqrt(sum((agent_state[:2] - robot_state[:2]) ** 2))
        if distance < safety_distance and distance > 0:
            idx.append(len(obstacle_states) + j)
    return idx


def rollout_cross_and_rescue(mod, steps):
    """cross_and_rescue.py:29-175 with single-integrator robots (rps absent):
    x_si := x, robots integrate p += T*u like the obstacles (:173); no si_barrier_cert."""
    c = mod.ControlBarrierFunction(15)
    N_robots, N_obs, diameter, T = 4, 6, 0.6, 1 / 30
    ic_r = np.zeros((N_robots, 3)); ic_o = np.zeros((N_obs, 2))
    center_obs = np.array([0, 0]); center_robots = np.array([0, 0, 0])
    for i in range(N_obs):
        theta = i * (2 * np.pi / N_obs)
        ic_o[i] = center_obs + [diameter * np.cos(theta), diameter * np.sin(theta)]
    for i in range(N_robots):
        theta = i * (2 * np.pi / N_robots)
        ic_r[i] = center_robots + [0.6 * diameter * np.cos(theta) - 1.15, 0.6 * diameter * np.sin(theta),
                                   theta + (2 / 3 * np.pi)]
    x = ic_r.T[:2].copy()
    obs_pos = ic_o.T.copy()
    L1 = np.array([[-1, 1, 0, 0, 0, 0], [0, -1, 1, 0, 0, 0], [0, 0, -1, 1, 0, 0], [0, 0, 0, -1, 1, 0],
                   [0, 0, 0, 0, -1, 1], [1, 0, 0, 0, 0, -1]])
    L2 = np.array([[-1, 0, 0, 0, 1], [1, -2, 0, 1, 0], [1, 1, -2, 0, 0], [1, 0, 1, -2, 0], [0, 0, 0, 0, 0]])
    rec = {k: [] for k in ("pos", "vel", "u", "nbr_mask", "pos_next", "relax_iters")}
    for _ in range(steps):
        x_si = np.concatenate((x, np.array([[1.5], [0]])), axis=1)
        si_velocities = np.zeros((2, N_robots)); obs_velocities = np.zeros((2, N_obs))
        for i in range(N_obs):
            j = topological_neighbors(L1, i)
            theta = -np.pi / N_obs
            rotation = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
            obs_velocities[:, i] = np.sum(obs_pos[:, j] - obs_pos[:, i, None], 1) @ rotation * 0.05
        for i in range(N_robots):
            j = topological_neighbors(L2, i)
            si_velocities[:, i] = np.sum(x_si[:, j] - x_si[:, i, None], 1)
        obs_pos_a = np.concatenate((obs_pos, np.zeros((2, 1))), axis=1)
        obs_vel_a = np.concatenate((obs_velocities, np.zeros((2, 1))), axis=1)
        obstacle_states = np.concatenate((obs_pos_a, obs_vel_a), axis=0).transpose()
        agent_states = np.concatenate((x[:2, :], si_velocities), axis=0).transpose()
        nbr_mask = np.zeros((N_robots, N_obs + 1 + N_robots), bool)
        its = np.zeros(N_robots, int)
        for i in range(N_robots):
            robot_state = agent_states[i]
            idx = cull(robot_state, obstacle_states, agent_states)
            nbr_mask[i, idx] = True
            if idx:
                allst = np.concatenate((obstacle_states, agent_states))
                sc = c.get_safe_control(robot_state, allst[idx], FX, GX,
                                        np.array([si_velocities[0][i], si_velocities[1][i]]))
                its[i] = _Recorder.calls[-1][3]
                si_velocities[0][i] = sc[0]; si_velocities[1][i] = sc[1]
        rec["pos"].append(np.concatenate((obs_pos_a, x), axis=1).T)
        rec["vel"].append(np.concatenate((obs_vel_a, agent_states[:, 2:].T), axis=1).T)
        rec["u"].append(si_velocities.T.copy())
        rec["nbr_mask"].append(nbr_mask); rec["relax_iters"].append(its)
        obs_pos = obs_pos_a[:, :N_obs] + T * obs_vel_a[:, :N_obs]         # :173
        x = x + T * si_velocities                                         # Euler stand-in for r.step()
        rec["pos_next"].append(np.concatenate((obs_pos, np.zeros((2, 1)), x), axis=1).T)
    return {k: np.array(v) for k, v in rec.items()}


def rollout_meet_at_center(mod, steps, N=10, gain=1.0):
    """meet_at_center.py:24-153 with single-integrator agents (rps absent); N=10 is the
    shipped geometry; N=100 is SURVEY cfg2 (gain 4/49 on the complete-graph consensus)."""
    c = mod.ControlBarrierFunction(15)
    half = N // 2
    diameter, T = 0.7, 1 / 30
    ic = np.zeros((N, 3)); center = np.array([0, 0, 0])
    for i in range(half):
        theta = i * (2 * np.pi / half)
        ic[i] = center + [diameter * np.cos(theta), diameter * np.sin(theta), theta + (2 / 3 * np.pi)]
    for i in range(half, N):
        theta = i * (2 * np.pi / half) + np.pi / 5
        ic[i] = center + [1.5 * diameter * np.cos(theta), 1.5 * diameter * np.sin(theta), theta + (2 / 3 * np.pi)]
    x = ic.T[:2].copy()
    L1 = np.zeros((half, half), int)
    for i in range(half):
        L1[i, i] = -1; L1[i, (i + 1) % half] = 1
    L2 = completeGL(half)
    rec = {k: [] for k in ("pos", "vel", "u", "nbr_mask", "pos_next", "relax_iters")}
    for _ in range(steps):
        x_si = x
        si_velocities = np.zeros((2, N))
        for i in range(half):
            j = topological_neighbors(L1, i)
            theta = -np.pi / half
            rotation = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
            si_velocities[:, i] = np.sum(x_si[:, j] - x_si[:, i, None], 1) @ rotation
        for i in range(half, N):
            j = topological_neighbors(L2, i - half) + half
            si_velocities[:, i] = np.sum(x_si[:, j] - x_si[:, i, None], 1) * gain
        states = np.concatenate((x[:2, :], si_velocities), axis=0).transpose()
        obstacle_states = states[:half]; agent_states = states[half:]
        nbr_mask = np.zeros((N - half, N), bool)
        its = np.zeros(N - half, int)
        vel = states[:, 2:].copy()
        for i in range(half, N):
            robot_state = states[i]
            idx = cull(robot_state, obstacle_states, agent_states)
            nbr_mask[i - half, idx] = True
            if idx:
                sc = c.get_safe_control(robot_state, states[idx], FX, GX,
                                        np.array([si_velocities[0][i], si_velocities[1][i]]))
                its[i - half] = _Recorder.calls[-1][3]
                si_velocities[0][i] = sc[0]; si_velocities[1][i] = sc[1]
        rec["pos"].append(x.T.copy()); rec["vel"].append(vel)
        rec["u"].append(si_velocities.T.copy()); rec["nbr_mask"].append(nbr_mask)
        rec["relax_iters"].append(its)
        x = x + T * si_velocities
        rec["pos_next"].append(x.T.copy())
    return {k: np.array(v) for k, v in rec.items()}


def consensus_vectors(rng):
    """np.sum(X[:, j] - X[:, i, None], 1) (+ '@ rotation * s') for degrees 1..40: pins the
    summation / gemv orders used by cross_and_rescue.py:118,125 and meet_at_center.py:96,103."""
    out = {"X": [], "deg": [], "theta": [], "scale": [], "plain": [], "rot": []}
    for deg in range(1, 41):
        for _ in range(8):
            X = rng.normal(0, 1, (2, deg + 1)) * (10 ** rng.uniform(-2, 1, (2, deg + 1)))
            j = np.arange(1, deg + 1)
            n = int(rng.integers(2, 60))
            theta = -np.pi / n
            scale = float(rng.choice([1.0, 0.05, 4 / 49, 0.25, 4 / 15]))
            rotation = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
            plain = np.sum(X[:, j] - X[:, 0, None], 1)
            rot = np.sum(X[:, j] - X[:, 0, None], 1) @ rotation * scale
            Xp = np.zeros((2, 41)); Xp[:, :deg + 1] = X
            out["X"].append(Xp); out["deg"].append(deg); out["theta"].append(theta)
            out["scale"].append(scale); out["plain"].append(plain); out["rot"].append(rot)
    return {k: np.array(v) for k, v in out.items()}


def main():
    mod = load_reference_cbf()
    rng = np.random.default_rng(20261015)
    fc = filter_cases(mod, rng)
    np.savez_compressed(os.path.join(HERE, "golden_filter.npz"), **fc)
    car = rollout_cross_and_rescue(mod, 400)
    print("cross_and_rescue: filter calls/step",
          car["nbr_mask"].any(axis=2).sum() / len(car["pos"]), "relaxed", (car["relax_iters"] != 0).sum())
    np.savez_compressed(os.path.join(HERE, "golden_cross_and_rescue.npz"), **car)
    mac = rollout_meet_at_center(mod, 300)
    print("meet_at_center N=10: filter calls/step", mac["nbr_mask"].any(axis=2).sum() / len(mac["pos"]),
          "relaxed", (mac["relax_iters"] != 0).sum())
    np.savez_compressed(os.path.join(HERE, "golden_meet_at_center.npz"), **mac)
    mac100 = rollout_meet_at_center(mod, 60, N=100, gain=4 / 49)
    print("meet_at_center N=100: filter calls/step", mac100["nbr_mask"].any(axis=2).sum() / len(mac100["pos"]),
          "relaxed", (mac100["relax_iters"] != 0).sum())
    np.savez_compressed(os.path.join(HERE, "golden_meet_at_center_n100.npz"), **mac100)
    cv = consensus_vectors(rng)
    np.savez_compressed(os.path.join(HERE, "golden_consensus.npz"), **cv)
    cl = {}
    t = 0.04
    s = [t]
    for _ in range(4):
        s.append(float(np.nextafter(s[-1], 1))); s.insert(0, float(np.nextafter(s[0], 0)))
    s = np.array(s + [0.0, 5e-324, 0.2 * 0.2])
    cl["s"] = s
    cl["keep"] = np.array([bool(np.sqrt(v) < 0.2) for v in s])
    np.savez_compressed(os.path.join(HERE, "golden_cull_threshold.npz"), **cl)


if __name__ == "__main__":
    main()
