"""The reference's CPU path timed on the host's cores, for bench.py's ``cpu_baseline`` leg.

TEST INFRASTRUCTURE ONLY (imported by bench.py's cpu_baseline leg and tests/, never by cbf_amd).

What is timed is ``oracle/refloop.py``: /root/reference/cross_and_rescue.py:135-160 restated line
by line (a Python cull over every entity per ego, the rows of cbf.py:38-80, cvxopt's coneqp of
cbf.py:75-87 restated in numpy since the cvxopt binary is absent, de-bias and clip).  Agents are
independent within a step (the loop is a Jacobi update over the packed nominal states,
cross_and_rescue.py:133), so the egos are split over one single-threaded process per host core
(OMP / OPENBLAS / MKL threads pinned to 1) and the rates add.

Shapes, each on the same inputs the GPU runs (plus ``cfg4_c``: the lattice egos through the C
restatement, oracle/cbf_oracle.c, SURVEY 8(d)'s second baseline):
  * ``qp``   -- cfg2 (meet_at_center.py:76-153 at N = 100: 50 pursuit obstacles, 50 agents), where
                the interior-point QP dominates each agent-QP;
  * ``cfg4`` -- random egos of a lattice (cfg4 / cfg4f / cfg4r at 1M agents, cfg3 at 65,536), where
                the reference's O(N) Python cull per ego dominates (that is what its loop does at
                that N);
  * ``mc``   -- cfg5: whole scenarios (16 agents against 32 entities each), QP-dominated.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def host_cores():
    """(cores, how) available to this job: the cgroup CPU quota, the affinity mask and the
    launcher's OMP_NUM_THREADS share, whichever is smallest (os.cpu_count() is the whole machine,
    which several GPU jobs share)."""
    cands = {}
    try:
        cands["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cands["cpu_count"] = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            cands["cgroup_quota"] = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        cands["OMP_NUM_THREADS"] = int(omp)
    how = min(cands, key=cands.get)
    return cands[how], f"{how}={cands[how]} (all: {cands}, machine cpu_count={os.cpu_count()})"


def _scenarios():
    """cbf_amd/scenarios.py (plain numpy) loaded by path: the package __init__ would load the HIP
    library into every worker process."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_cbf_scenarios", os.path.join(ROOT, "cbf_amd", "scenarios.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pin_blas():
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"


def _cfg2_state():
    """cfg2's packed states at step 0: positions and nominal controls (meet_at_center.py:86-116)."""
    from oracle import coracle
    pos, n_obs, groups = _scenarios().meet_at_center(100)
    vel = np.zeros_like(pos)
    for (b, e, rows, anc, rot, scale) in groups:
        rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
        col = np.array([j for r in rows for j in r], np.int32)
        vel[b:e] = coracle.consensus_csr(pos[b:e], rp, col, 0, e - b, anchors=anc, rot=rot, scale=scale)
    return pos, vel, n_obs


def _cfg4_state(W, H, seed, spacing, gain, nominal=None):
    """The lattice at step 0 with its nominal controls: the lattice Laplacian (cfg4 / cfg4f /
    cfg3) or cfg4r's random walk (pyoracle.random_nominal)."""
    from oracle import coracle, pyoracle as po
    pos = _scenarios().lattice(W, H, seed=seed, spacing=spacing)
    if nominal is not None:
        _, amp, nseed = nominal
        return pos, po.random_nominal(pos, 0, amp, nseed), 0
    return pos, coracle.consensus_lattice(W, H, 0, H, pos, gain), 0


def _mc_state(all_pos, gain, s):
    """cfg5 scenario s at step 0 (scenarios.mc_scenarios: 16 pursuit obstacles + 16 free agents)
    with its nominal controls: cyclic pursuit of the obstacles (rotation -pi/16, meet_at_center.py:
    86-96) and the complete-graph consensus of the agents with the cfg5 gain (:99-103)."""
    from oracle import coracle
    pos = np.ascontiguousarray(all_pos[s])
    ring = [[(i + 1) % 16] for i in range(16)]
    full = [[j for j in range(16) if j != i] for i in range(16)]
    th = -np.pi / 16
    vel = np.zeros_like(pos)
    for (b, e, rows, rot, scale) in ((0, 16, ring, (np.cos(th), np.sin(th)), 1.0), (16, 32, full, None, gain)):
        rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
        col = np.array([j for r in rows for j in r], np.int32)
        vel[b:e] = coracle.consensus_csr(pos[b:e], rp, col, 0, e - b, rot=rot, scale=scale)
    return pos, vel, 16


def _c_loop(pos, vel, egos, budget_s):
    """The same loop in the C restatement (oracle/cbf_oracle.c: the reference's O(N) cull per ego,
    rows, the exact 2-D QP with the +1 rule, clip): SURVEY 8(d)'s second CPU baseline."""
    from oracle import coracle, pyoracle as po
    p = po.Params(15)
    t0 = time.perf_counter()
    done = solves = 0
    for e in egos:
        if time.perf_counter() - t0 >= budget_s:
            break
        out = coracle.filter_swarm(p, pos, vel, 0, e, e + 1)
        solves += int(out["cnt"][0] > 0)
        done += 1
    return done, solves, time.perf_counter() - t0


def _worker(arg):
    kind, shape, rank, procs, budget_s = arg
    _pin_blas()
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import pyoracle as po, refloop
    if kind == "mc":   # scenarios rank, rank + procs, ...: each one loop over its 16 agents
        # scenario states at timestep t_state of the GPU rollout (step 0 has no neighbour within
        # the cull radius), rolled forward by the C restatement (not timed)
        n_scen, seed, gain, t_state = shape
        from oracle import coracle
        all_pos = _scenarios().mc_scenarios(n_scen, 16, 16, seed=seed)   # the GPU run's batch
        th = -np.pi / 16
        done = solves = 0
        spent = 0.0   # seconds in the reference loop only
        for sc in range(rank, n_scen, procs):
            left = budget_s - spent
            if left <= 0:
                break
            rolled = coracle.mc_rollout(po.Params(15), all_pos[sc:sc + 1], 16, 16, t_state, 1 / 30,
                                        (np.cos(th), np.sin(th)), 1.0, gain)[0]
            pos, vel, n_obs = _mc_state(rolled, gain, 0)
            d, s, dt = refloop.loop_sample(po.Params(15), pos, vel, n_obs, range(16), left)
            done += d
            solves += s
            spent += dt
        return done, solves, spent
    if kind == "cfg4_c":
        pos, vel, _ = _cfg4_state(*shape)
        order = np.random.default_rng(321).permutation(pos.shape[0])
        return _c_loop(pos, vel, (int(e) for e in order[rank::procs]), budget_s)
    if kind == "qp":
        pos, vel, n_obs = _cfg2_state()
        n_ego = pos.shape[0] - n_obs
        egos = (i % n_ego for i in range(rank, 1 << 40, procs))        # the 50 agents, cyclically
    else:
        pos, vel, n_obs = _cfg4_state(*shape)
        order = np.random.default_rng(321).permutation(pos.shape[0] - n_obs)
        egos = (int(e) for e in order[rank::procs])
    done, solves, dt = refloop.loop_sample(po.Params(15), pos, vel, n_obs, egos, budget_s)
    return done, solves, dt


def run(kind, budget_s, procs=None, shape=None):
    """Times the restated reference loop on `procs` processes (default: host_cores()) for about
    budget_s seconds each.  Returns the cpu_baseline record."""
    cores, how = host_cores()
    procs = procs or cores
    args = [(kind, shape, r, procs, budget_s) for r in range(procs)]
    t0 = time.perf_counter()
    # close + join (not the `with` block's terminate): the workers exit on their own, so no
    # SIGTERM traces land in a profiler's log
    pool = mp.get_context("spawn").Pool(procs)
    try:
        res = pool.map(_worker, args)
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    wall = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    solves = sum(r[1] for r in res)
    dt = max(r[2] for r in res)
    if kind == "cfg4_c":
        return {"value": solves / dt, "unit": "agent-QP solves/s", "cores": procs, "kind": "port",
                "per_core": solves / dt / procs,
                "sample": f"{done} random egos of the {shape[0]}x{shape[1]} lattice (spacing {shape[3]}) through the "
                          f"C restatement oracle/cbf_oracle.c (the reference's O(N) cull per ego, cbf.py rows, the "
                          f"exact 2-D QP with the +1 rule, clip), {procs} single-threaded processes x {dt:.1f} s",
                "cores_source": how}
    if kind == "qp":
        what = ("cfg2 (meet_at_center.py at N=100: 50 obstacles + 50 agents, step-0 states), every agent-QP "
                "one cvxopt-coneqp solve")
    elif kind == "mc":
        what = (f"cfg5 scenarios (of {shape[0]}; 16 pursuit obstacles + 16 agents each, states at timestep "
                f"{shape[3]} of the rollout, meet_at_center.py:118-143 per scenario), each agent a 32-entity Python "
                "cull + cvxopt-coneqp solve (the rollout to that timestep by the C restatement, untimed, is "
                "excluded from the rate)")
    else:
        nom = "" if len(shape) < 6 or shape[5] is None else ", random-walk nominal control"
        what = (f"random egos of the {shape[0]}x{shape[1]} lattice (spacing {shape[3]}{nom}), each an O(N) "
                "Python cull + cvxopt-coneqp solve")
    from oracle import refloop
    return {"value": solves / dt, "unit": "agent-QP solves/s", "cores": procs, "kind": "port",
            "per_core": solves / dt / procs,
            "qp_solver": refloop.QP_SOLVER,
            "sample": f"{done} egos of {what}, through oracle/refloop.py (cross_and_rescue.py:135-160 restated "
                      f"line by line; QP: {refloop.QP_SOLVER}, maxiters 600), {procs} single-threaded processes "
                      f"x {dt:.1f} s ({wall:.1f} s wall incl. start-up)",
            "cores_source": how}
