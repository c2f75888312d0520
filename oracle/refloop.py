"""Line-by-line Python restatement of the reference's per-agent CPU loop, for the bench's
``cpu_baseline`` leg.  TEST INFRASTRUCTURE ONLY (never imported by ``cbf_amd``).

/root/reference/cross_and_rescue.py:135-160 (same shape in meet_at_center.py:118-143): for every
robot, a Python loop over all obstacles and then all agents evaluating
``np.sqrt(sum((s[:2] - robot_state[:2])**2))``, the neighbour list as a Python list, and -- when it
is non-empty -- ``get_safe_control`` (cbf.py:18-92): the rows of cbf.py:38-80 (pyoracle.assemble,
bit-exact to the reference) handed to cvxopt's QP (restated in oracle/cvxqp.py, since the cvxopt
binary is absent), then de-bias and clip.  It is what the reference's CPU path costs per
agent-QP, up to cvxopt's C-level BLAS calls versus numpy's.
"""
from __future__ import annotations

import time
import warnings

import numpy as np

from . import cvxqp
from . import pyoracle as po

# the real cvxopt binary is used when the box has it (it is absent from this
# image); otherwise the numpy restatement of its coneqp (oracle/cvxqp.py).
try:
    import cvxopt as _cvxopt
    QP_SOLVER = f"cvxopt {getattr(_cvxopt, '__version__', '?')} (solvers.qp)"
except ImportError:
    _cvxopt = None
    QP_SOLVER = "cvxopt coneqp restated in numpy (oracle/cvxqp.py; the cvxopt binary is absent)"


def _cvxopt_safe_control(A, b, m, u0, max_speed):
    """cbf.py:64-92 through the cvxopt binary: min 1/2 |x|^2 s.t. A x <= b, every barrier rhs +1
    while the solver raises ValueError, then de-bias and clip."""
    M = _cvxopt.matrix
    _cvxopt.solvers.options["show_progress"] = False                  # cbf.py:75-76
    _cvxopt.solvers.options["maxiters"] = 600
    P, q = M(np.eye(2)), M(np.zeros((2, 1)))
    b = np.array(b, dtype=np.float64).reshape(-1, 1)
    while True:
        try:
            x = np.array(_cvxopt.solvers.qp(P, q, M(np.asarray(A, dtype=np.float64)), M(b))["x"]).reshape(2)
            break
        except ValueError:                                             # cbf.py:84-87
            b[:m] += 1
    u = x + np.asarray(u0, dtype=np.float64).reshape(2)
    return np.array([max(min(u[0], max_speed), -max_speed), max(min(u[1], max_speed), -max_speed)])


def get_safe_control(p: po.Params, robot_state, danger, u0):
    A, b = po.assemble(p, robot_state, danger, u0)                    # cbf.py:38-80
    if _cvxopt is not None:
        return _cvxopt_safe_control(A, b, len(danger), u0, p.max_speed)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        u, _ = cvxqp.get_safe_control(A, b, len(danger), u0, p.max_speed)  # cbf.py:75-92
    return u


def loop_sample(p: po.Params, pos, vel, n_obs, egos, budget_s, safety_distance=0.2):
    """Runs the reference loop body for the agents in ``egos`` (indices among the agents) until
    ``budget_s`` has elapsed.  Returns (egos done, agent-QP solves, seconds)."""
    states = np.concatenate([np.asarray(pos), np.asarray(vel)], axis=1)   # cross_and_rescue.py:132-133
    obstacle_states, agent_states = states[:n_obs], states[n_obs:]
    t0 = time.perf_counter()
    done = solves = 0
    for i in egos:
        if time.perf_counter() - t0 >= budget_s:
            break
        danger_obstacle_states = []
        robot_state = agent_states[i]
        for obstacle_state in obstacle_states:                             # :141-144
            distance = np.sqrt(sum((obstacle_state[:2] - robot_state[:2]) ** 2))
            if distance < safety_distance:
                danger_obstacle_states.append(obstacle_state)
        for agent_state in agent_states:                                   # :147-150
            distance = np.sqrt(sum((agent_state[:2] - robot_state[:2]) ** 2))
            if distance < safety_distance and distance > 0:
                danger_obstacle_states.append(agent_state)
        if len(danger_obstacle_states) > 0:                                # :153-160
            get_safe_control(p, robot_state, np.array(danger_obstacle_states), robot_state[2:4])
            solves += 1
        done += 1
    return done, solves, time.perf_counter() - t0
