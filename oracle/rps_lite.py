"""CPU restatement of the robotarium (``rps``) pieces the reference scripts call around the filter.

TEST INFRASTRUCTURE ONLY (the checker: imported by ``tests/`` and never by ``cbf_amd``).

SURVEY.md 8(f) rows 2-3.  The reference scripts import ``rps`` (robotarium_python_simulator),
a third-party package that ``/root/reference/install.sh:1`` clones at an unpinned HEAD and that
is absent from this image (``robotarium_python_simulator/`` is empty).  What the scripts call:

* ``create_si_to_uni_mapping()``              cross_and_rescue.py:75, meet_at_center.py:61
    -> ``uni_to_si_states(x)``                  cross_and_rescue.py:101, meet_at_center.py:80
    -> ``si_to_uni_dyn(dxi, x)``                cross_and_rescue.py:167, meet_at_center.py:148
* ``create_single_integrator_barrier_certificate_with_boundary(safety_radius=0.12)``
                                              cross_and_rescue.py:72 (applied :163);
                                              meet_at_center.py:58 (application commented out :109)
* ``Robotarium.set_velocities`` / ``step``      cross_and_rescue.py:170,175; meet_at_center.py:151,153

Each function below restates the published robotarium_python_simulator algorithm
(``rps/utilities/transformations.py``, ``rps/utilities/barrier_certificates.py``,
``rps/robotarium_abc.py``, ``rps/robotarium.py``) from its documented behaviour.  No reference
test or fixture pins any of it: **parity unpinned** (DESIGN.md).  The coupled barrier-certificate
QP is solved here exactly (Goldfarb-Idnani dual active set, certified by KKT residuals in the
tests) and, for comparison, by the restated cvxopt ``coneqp`` (oracle/cvxqp.py) with the solver
options rps sets at import (reltol = feastol = 1e-2, maxiters 50 -- upstream, unverified).
"""
from __future__ import annotations

import math

import numpy as np

# rps/robotarium_abc.py constants [upstream, unverified]
TIME_STEP = 0.033
ROBOT_DIAMETER = 0.11
WHEEL_RADIUS = 0.016
BASE_LENGTH = 0.105
MAX_LINEAR_VELOCITY = 0.2
MAX_ANGULAR_VELOCITY = 2 * (WHEEL_RADIUS / ROBOT_DIAMETER) * (MAX_LINEAR_VELOCITY / WHEEL_RADIUS)
MAX_WHEEL_VELOCITY = MAX_LINEAR_VELOCITY / WHEEL_RADIUS

# create_si_to_uni_mapping defaults
PROJECTION_DISTANCE = 0.05
ANGULAR_VELOCITY_LIMIT = np.pi

# create_single_integrator_barrier_certificate_with_boundary defaults
BARRIER_GAIN = 100
SAFETY_RADIUS = 0.17
MAGNITUDE_LIMIT = 0.2
BOUNDARY_POINTS = (-1.6, 1.6, -1.0, 1.0)

# status of the coupled QP
CERT_OPTIMAL = 1
CERT_INFEASIBLE = 2   # empty polyhedron: the thresholded input is returned
CERT_MAXITER = 3


# ------------------------------------------------------------------------------------------
# si <-> uni maps (transformations.py create_si_to_uni_mapping)
# ------------------------------------------------------------------------------------------
def uni_to_si_states(poses, projection_distance=PROJECTION_DISTANCE):
    """(3, N) unicycle poses -> (2, N) projection points x + l (cos th, sin th)
    (cross_and_rescue.py:101)."""
    poses = np.asarray(poses, dtype=np.float64)
    si = np.zeros((2, poses.shape[1]))
    si[0, :] = poses[0, :] + projection_distance * np.cos(poses[2, :])
    si[1, :] = poses[1, :] + projection_distance * np.sin(poses[2, :])
    return si


def si_to_uni_dyn(dxi, poses, projection_distance=PROJECTION_DISTANCE, angular_velocity_limit=ANGULAR_VELOCITY_LIMIT):
    """(2, N) single-integrator velocities at the projection points -> (2, N) unicycle (v, w),
    w clamped to +-angular_velocity_limit (cross_and_rescue.py:167)."""
    dxi = np.asarray(dxi, dtype=np.float64)
    poses = np.asarray(poses, dtype=np.float64)
    cs = np.cos(poses[2, :])
    ss = np.sin(poses[2, :])
    dxu = np.zeros((2, dxi.shape[1]))
    dxu[0, :] = cs * dxi[0, :] + ss * dxi[1, :]
    dxu[1, :] = (1 / projection_distance) * (-ss * dxi[0, :] + cs * dxi[1, :])
    dxu[1, dxu[1, :] > angular_velocity_limit] = angular_velocity_limit
    dxu[1, dxu[1, :] < -angular_velocity_limit] = -angular_velocity_limit
    return dxu


# ------------------------------------------------------------------------------------------
# Robotarium.set_velocities / step (robotarium_abc.py, robotarium.py)
# ------------------------------------------------------------------------------------------
def set_velocities(dxu):
    """Linear / angular saturation of set_velocities (cross_and_rescue.py:170)."""
    v = np.array(dxu, dtype=np.float64)
    i = np.abs(v[0, :]) > MAX_LINEAR_VELOCITY
    v[0, i] = MAX_LINEAR_VELOCITY * np.sign(v[0, i])
    i = np.abs(v[1, :]) > MAX_ANGULAR_VELOCITY
    v[1, i] = MAX_ANGULAR_VELOCITY * np.sign(v[1, i])
    return v


def wheel_threshold(dxu):
    """step()'s motor thresholding: unicycle -> wheel speeds, clamp to the max wheel speed, back."""
    r, l = WHEEL_RADIUS, BASE_LENGTH
    dxu = np.asarray(dxu, dtype=np.float64)
    dxdd = np.vstack((1 / (2 * r) * (2 * dxu[0, :] - l * dxu[1, :]), 1 / (2 * r) * (2 * dxu[0, :] + l * dxu[1, :])))
    t = np.absolute(dxdd) > MAX_WHEEL_VELOCITY
    dxdd[t] = MAX_WHEEL_VELOCITY * np.sign(dxdd[t])
    return np.vstack((r / 2 * (dxdd[0, :] + dxdd[1, :]), r / l * (dxdd[1, :] - dxdd[0, :])))


def unicycle_step(poses, velocities, dt=TIME_STEP):
    """Robotarium.step(): threshold motors, Euler on (x, y, theta), wrap theta with atan2
    (cross_and_rescue.py:175)."""
    p = np.array(poses, dtype=np.float64)
    v = wheel_threshold(velocities)
    p[0, :] = p[0, :] + dt * np.cos(p[2, :]) * v[0, :]
    p[1, :] = p[1, :] + dt * np.sin(p[2, :]) * v[0, :]
    p[2, :] = p[2, :] + dt * v[1, :]
    p[2, :] = np.arctan2(np.sin(p[2, :]), np.cos(p[2, :]))
    return p


# ------------------------------------------------------------------------------------------
# single-integrator barrier certificate with boundary (barrier_certificates.py)
# ------------------------------------------------------------------------------------------
def si_barrier_qp(dxi, x, barrier_gain=BARRIER_GAIN, safety_radius=SAFETY_RADIUS, magnitude_limit=MAGNITUDE_LIMIT,
                  boundary_points=BOUNDARY_POINTS):
    """The QP of si_barrier_cert(dxi, x) (cross_and_rescue.py:163): returns (y, A, b) with y the
    magnitude-thresholded input (2N, x-major per agent) and A y' <= b the rows in rps order --
    every pair i < j (lexicographic), then per agent: +y, -y, +x, -x boundary rows.  The QP is
    min 1/2 v'(2I)v - 2 y'v  s.t.  A v <= b, i.e. the projection of y onto {A v <= b}."""
    dxi = np.array(dxi, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    N = dxi.shape[1]
    m = N * (N - 1) // 2 + 4 * N
    A = np.zeros((m, 2 * N))
    b = np.zeros(m)
    c = 0
    for i in range(N - 1):
        for j in range(i + 1, N):
            e = x[:, i] - x[:, j]
            h = (e[0] * e[0] + e[1] * e[1]) - np.power(safety_radius, 2)
            A[c, (2 * i, 2 * i + 1)] = -2 * e
            A[c, (2 * j, 2 * j + 1)] = 2 * e
            b[c] = barrier_gain * np.power(h, 3)
            c += 1
    bp = boundary_points
    for k in range(N):
        A[c, (2 * k, 2 * k + 1)] = np.array([0, 1])
        b[c] = 0.4 * barrier_gain * np.power(bp[3] - safety_radius / 2 - x[1, k], 3)
        c += 1
        A[c, (2 * k, 2 * k + 1)] = -np.array([0, 1])
        b[c] = 0.4 * barrier_gain * np.power(-bp[2] - safety_radius / 2 + x[1, k], 3)
        c += 1
        A[c, (2 * k, 2 * k + 1)] = np.array([1, 0])
        b[c] = 0.4 * barrier_gain * np.power(bp[1] - safety_radius / 2 - x[0, k], 3)
        c += 1
        A[c, (2 * k, 2 * k + 1)] = -np.array([1, 0])
        b[c] = 0.4 * barrier_gain * np.power(-bp[0] - safety_radius / 2 + x[0, k], 3)
        c += 1
    norms = np.linalg.norm(dxi, 2, 0)
    idx = norms > magnitude_limit
    dxi[:, idx] *= magnitude_limit / norms[idx]
    y = np.reshape(dxi, 2 * N, order="F")
    return y, A, b


def goldfarb_idnani(y, A, b, max_iter=None, viol_tol=1e-12):
    """Exact projection of y onto {v : A v <= b} (min |v - y|^2) by the Goldfarb-Idnani dual
    active-set method (Math. Programming 27, 1983) for the Hessian 2I: J = L^-T Q with
    L = sqrt(2) I, R the triangular factor of the active normals, Givens updates on add / drop.

    Returns dict(x, status, active (row indices), lam (their multipliers), iters)."""
    y = np.asarray(y, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    n, m = y.shape[0], A.shape[0]
    max_iter = max_iter or 10 * (m + n) + 10
    x = y.copy()
    J = np.eye(n) / math.sqrt(2.0)
    R = np.zeros((n, n))
    act, u = [], []
    q = 0
    it = 0

    def slack(i, xv):
        return b[i] - A[i] @ xv

    def drop(k):
        nonlocal q
        # delete column k of R, restore the triangle with Givens on rows (j, j+1), same on J
        for j in range(k, q - 1):
            R[:, j] = R[:, j + 1]
        R[:, q - 1] = 0.0
        for j in range(k, q - 1):
            a_, b_ = R[j, j], R[j + 1, j]
            h = math.hypot(a_, b_)
            if h == 0.0:
                continue
            c, s = a_ / h, b_ / h
            Rj, Rj1 = R[j, :].copy(), R[j + 1, :].copy()
            R[j, :] = c * Rj + s * Rj1
            R[j + 1, :] = -s * Rj + c * Rj1
            R[j + 1, j] = 0.0
            Jj, Jj1 = J[:, j].copy(), J[:, j + 1].copy()
            J[:, j] = c * Jj + s * Jj1
            J[:, j + 1] = -s * Jj + c * Jj1
        del act[k]
        del u[k]
        q -= 1

    while True:
        it += 1
        if it > max_iter:
            return dict(x=x, status=CERT_MAXITER, active=list(act), lam=list(u), iters=it)
        s = b - A @ x
        s_act = s.copy()
        s_act[act] = np.inf
        p = int(np.argmin(s_act)) if m else -1
        if m == 0 or not (s_act[p] < -viol_tol * max(1.0, abs(b[p]))):
            return dict(x=x, status=CERT_OPTIMAL, active=list(act), lam=list(u), iters=it)
        npl = -A[p]            # normal of the constraint b_p - A_p v >= 0
        up = 0.0
        while True:
            d = J.T @ npl
            z = J[:, q:] @ d[q:]
            r = np.zeros(q)
            for j in reversed(range(q)):        # R r = d[:q]
                r[j] = (d[j] - R[j, j + 1:q] @ r[j + 1:q]) / R[j, j]
            t1, k = math.inf, -1
            for j in range(q):
                if r[j] > 0.0:
                    tj = u[j] / r[j]
                    if tj < t1:
                        t1, k = tj, j
            zn = float(d[q:] @ d[q:])           # z' n+ = |d2|^2
            if zn > 1e-28 * float(d @ d):
                t2 = -slack(p, x) / zn          # c_p(x + t z) = slack + t z'n+ = 0
            else:
                t2 = math.inf
            if t1 == math.inf and t2 == math.inf:
                return dict(x=x, status=CERT_INFEASIBLE, active=list(act), lam=list(u), iters=it)
            if t2 == math.inf:
                for j in range(q):
                    u[j] -= t1 * r[j]
                up += t1
                drop(k)
                continue
            t = min(t1, t2)
            x = x + t * z
            for j in range(q):
                u[j] -= t * r[j]
            up += t
            if t2 <= t1:
                # add p: rotate d[q:] onto e_q (bottom up), same rotations on J's columns
                for j in range(n - 1, q, -1):
                    a_, b_ = d[j - 1], d[j]
                    if b_ == 0.0:
                        continue
                    h = math.hypot(a_, b_)
                    c, s_ = a_ / h, b_ / h
                    d[j - 1], d[j] = h, 0.0
                    Jc, Jc1 = J[:, j - 1].copy(), J[:, j].copy()
                    J[:, j - 1] = c * Jc + s_ * Jc1
                    J[:, j] = -s_ * Jc + c * Jc1
                R[:q + 1, q] = d[:q + 1]
                act.append(p)
                u.append(up)
                q += 1
                break
            drop(k)                             # partial step: constraint k left the active set


def si_barrier_cert(dxi, x, barrier_gain=BARRIER_GAIN, safety_radius=SAFETY_RADIUS, magnitude_limit=MAGNITUDE_LIMIT,
                    boundary_points=BOUNDARY_POINTS):
    """si_barrier_cert(dxi, x) (cross_and_rescue.py:163) solved exactly.  Returns ((2, N) result, info).
    An infeasible QP returns the thresholded input with status CERT_INFEASIBLE."""
    N = np.shape(dxi)[1]
    y, A, b = si_barrier_qp(dxi, x, barrier_gain, safety_radius, magnitude_limit, boundary_points)
    res = goldfarb_idnani(y, A, b)
    v = res["x"] if res["status"] == CERT_OPTIMAL else y
    res.update(y=y, A=A, b=b)
    return np.reshape(v, (2, N), order="F"), res


def kkt_residuals(y, A, b, x, active, lam):
    """(primal violation, stationarity |2(x - y) + A_act' lam|, min lam, complementarity)."""
    A = np.asarray(A)
    b = np.asarray(b)
    viol = float(max(0.0, np.max(A @ x - b))) if len(b) else 0.0
    g = 2.0 * (x - y)
    for i, l in zip(active, lam):
        g = g + l * A[i]
    stat = float(np.max(np.abs(g))) if len(g) else 0.0
    lmin = float(min(lam)) if lam else 0.0
    comp = float(max((abs(l * (b[i] - A[i] @ x)) for i, l in zip(active, lam)), default=0.0))
    return viol, stat, lmin, comp


# ------------------------------------------------------------------------------------------
# cross_and_rescue.py as shipped: unicycle robots + si_barrier_cert (cfg1 with rps-lite)
# ------------------------------------------------------------------------------------------
def cross_and_rescue_initial():
    """cross_and_rescue.py:36-57: robot poses (3, 4) and obstacle positions (2, 6)."""
    N_robots, N_obs, diameter = 4, 6, 0.6
    ic_r = np.zeros((N_robots, 3))
    ic_o = np.zeros((N_obs, 2))
    for i in range(N_obs):
        th = i * (2 * np.pi / N_obs)
        ic_o[i] = np.array([0, 0]) + [diameter * np.cos(th), diameter * np.sin(th)]
    for i in range(N_robots):
        th = i * (2 * np.pi / N_robots)
        ic_r[i] = np.array([0, 0, 0]) + [0.6 * diameter * np.cos(th) - 1.15, 0.6 * diameter * np.sin(th),
                                         th + (2 / 3 * np.pi)]
    return ic_r.T.copy(), ic_o.T.copy()


def cross_and_rescue_step(poses, obs_pos, params, T=1 / 30, safety_radius=0.12):
    """One iteration of cross_and_rescue.py:97-175 with rps-lite: returns (poses', obs_pos', rec).
    The per-robot CBF filter is the exact oracle (pyoracle.filter_one), the post-filter is
    si_barrier_cert solved exactly."""
    from . import pyoracle as po
    N_robots, N_obs = poses.shape[1], obs_pos.shape[1]
    x = poses
    x_si = uni_to_si_states(x)                                                   # :101
    x_si = np.concatenate((x_si, np.array([[1.5], [0]])), axis=1)                # :102
    si_velocities = np.zeros((2, N_robots))
    obs_velocities = np.zeros((2, N_obs))
    theta = -np.pi / N_obs
    rotation = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
    for i in range(N_obs):                                                       # :108-118 (L1 ring)
        j = [(i + 1) % N_obs]
        obs_velocities[:, i] = np.sum(obs_pos[:, j] - obs_pos[:, i, None], 1) @ rotation * 0.05
    l2 = [[4], [0, 3], [0, 1], [0, 2]]                                           # :89-95 rows 0..3
    for i in range(N_robots):                                                    # :121-125
        si_velocities[:, i] = np.sum(x_si[:, l2[i]] - x_si[:, i, None], 1)
    nominal = si_velocities.copy()
    obs_pos_a = np.concatenate((obs_pos, np.zeros((2, 1))), axis=1)              # :130
    obs_vel_a = np.concatenate((obs_velocities, np.zeros((2, 1))), axis=1)       # :131
    pos_all = np.concatenate((obs_pos_a, x[:2, :]), axis=1).T                    # :132-133
    vel_all = np.concatenate((obs_vel_a, si_velocities), axis=1).T
    u, status, cnt, _ = po.filter_swarm(params, pos_all, vel_all, N_obs + 1, N_obs + 1, N_obs + 1 + N_robots)
    si_velocities = u.T.copy()                                                   # :158-160
    filtered = si_velocities.copy()
    si_velocities, info = si_barrier_cert(si_velocities, x_si[:, :N_robots], safety_radius=safety_radius)  # :163
    dxu = si_to_uni_dyn(si_velocities, x)                                        # :167
    dxu = set_velocities(dxu)                                                    # :170
    obs_next = obs_pos_a[:, :N_obs] + T * obs_vel_a[:, :N_obs]                   # :173
    poses_next = unicycle_step(x, dxu)                                           # :175
    rec = dict(nominal=nominal, filtered=filtered, status=status, cnt=cnt, cert=si_velocities, dxu=dxu,
               cert_status=info["status"])
    return poses_next, obs_next, rec


# ------------------------------------------------------------------------------------------
# meet_at_center.py as shipped: N unicycle robots (half pursuit obstacles), no certificate
# ------------------------------------------------------------------------------------------
def meet_at_center_initial(N=10):
    """meet_at_center.py:37-48 (written for N = 10: 5 obstacles on radius 0.7, 5 agents on 1.05)."""
    half = N // 2
    ic = np.zeros((N, 3))
    diameter = 0.7
    for i in range(half):
        th = i * (2 * np.pi / half)
        ic[i] = np.array([0, 0, 0]) + [diameter * np.cos(th), diameter * np.sin(th), th + (2 / 3 * np.pi)]
    for i in range(half, N):
        th = i * (2 * np.pi / half) + np.pi / 5
        ic[i] = np.array([0, 0, 0]) + [1.5 * diameter * np.cos(th), 1.5 * diameter * np.sin(th),
                                       th + (2 / 3 * np.pi)]
    return ic.T.copy()


def meet_at_center_step(poses, params, gain=1.0):
    """One iteration of meet_at_center.py:76-153 with rps-lite: cyclic pursuit of the first N/2
    robots on the projection points (L1 ring, rotation -pi/(N/2)), complete-graph consensus of
    the rest (x gain; the script has gain 1), the CBF filter of every free robot against all
    obstacle robots and the other free robots (raw poses, Jacobi), si_to_uni_dyn ->
    set_velocities -> unicycle step for every robot (the certificate is commented out, :109)."""
    from . import pyoracle as po
    N = poses.shape[1]
    half = N // 2
    x = poses
    x_si = uni_to_si_states(x)                                                   # :80
    si_velocities = np.zeros((2, N))
    theta = -np.pi / half
    rotation = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
    for i in range(half):                                                        # :86-96
        j = [(i + 1) % half]
        si_velocities[:, i] = np.sum(x_si[:, j] - x_si[:, i, None], 1) @ rotation
    for i in range(half, N):                                                     # :99-103
        j = [q for q in range(half, N) if q != i]
        v = np.sum(x_si[:, j] - x_si[:, i, None], 1)
        si_velocities[:, i] = v if gain == 1.0 else v * gain
    nominal = si_velocities.copy()
    states = np.concatenate((x[:2, :], si_velocities), axis=0).transpose()      # :114
    u, status, cnt, _ = po.filter_swarm(params, states[:, :2], states[:, 2:], half, half, N)  # :117-143
    si_velocities[:, half:] = u.T
    dxu = si_to_uni_dyn(si_velocities, x)                                        # :148
    dxu = set_velocities(dxu)                                                    # :151
    poses_next = unicycle_step(x, dxu)                                           # :153
    return poses_next, dict(nominal=nominal, filtered=si_velocities.copy(), status=status, cnt=cnt, dxu=dxu)
