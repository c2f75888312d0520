"""HIP path (through the C ABI) against the golden vectors captured from the reference and the
CPU oracle.  Bars: integer/index results bit-exact; controls bit-exact vs the oracle (same
arithmetic) and within 1e-12 of the golden KKT-certified minimisers."""
import concurrent.futures as cf

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU boxes but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

import cbf_amd  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402
from oracle import coracle, pyoracle as po  # noqa: E402
from tests import paramsets  # noqa: E402

DEV = torch.device("cuda")
GX = 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]])


def _t(a, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=DEV)


def _golden_groups(F):
    """Group golden filter cases by parameter set -> one batched launch per group."""
    keys = {}
    for i in range(len(F["r"])):
        key = (float(F["max_speed"][i]), float(F["dmin"][i]), float(F["k"][i]), F["g"][i].tobytes(),
               F["f"][i].tobytes())
        keys.setdefault(key, []).append(i)
    return keys


def test_get_safe_control_batch_vs_golden(golden):
    F = golden("golden_filter.npz")
    cbf = cbf_amd.ControlBarrierFunction(15)
    n_checked = 0
    for (ms, dmin, k, gb, fb), idx in _golden_groups(F).items():
        g = np.frombuffer(gb, dtype=np.float64).reshape(4, 2)
        f = np.frombuffer(fb, dtype=np.float64).reshape(4, 4)
        c = cbf_amd.ControlBarrierFunction(ms, dmin=dmin, k=k)
        obs = [F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]] for i in idx]
        off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int32)
        u, st, x = c.get_safe_control_batch(_t(F["r"][idx]), (_t(off, torch.int32), _t(np.vstack(obs))),
                                            _t(F["u0"][idx]), f=f, g=g, return_x=True)
        u, st, x = u.cpu().numpy(), st.cpu().numpy(), x.cpu().numpy()
        p = po.Params(ms, dmin, k, g=g, f=f)
        for t, i in enumerate(idx):
            it = int(F["relax_iters"][i])
            want = po.STATUS_OPTIMAL if it == 0 else (po.STATUS_RELAXED if it > 0 else po.STATUS_BOX_INFEASIBLE)
            assert st[t] & 0xFF == want, i
            if it > 0:
                assert st[t] >> 8 == it, i
            assert np.abs(x[t] - F["x"][i]).max() <= 1e-12, i
            assert np.abs(u[t] - F["u"][i]).max() <= 1e-12, i
            ref = coracle.filter_one(p, F["r"][i], obs[t], F["u0"][i])
            assert np.array_equal(u[t], ref["u"]) and np.array_equal(x[t], ref["x"]), i
            n_checked += 1
    assert n_checked == len(F["r"])
    del cbf


def test_assemble_rows_bit_exact_vs_reference(golden):
    F = golden("golden_filter.npz")
    for (ms, dmin, k, gb, fb), idx in _golden_groups(F).items():
        g = np.frombuffer(gb, dtype=np.float64).reshape(4, 2)
        f = np.frombuffer(fb, dtype=np.float64).reshape(4, 4)
        c = cbf_amd.ControlBarrierFunction(ms, dmin=dmin, k=k)
        obs = [F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]] for i in idx]
        off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int32)
        A, b = c.assemble_rows(_t(F["r"][idx]), _t(off, torch.int32), _t(np.vstack(obs)), _t(F["u0"][idx]),
                               f=f, g=g)
        A, b = A.cpu().numpy(), b.cpu().numpy()
        for t, i in enumerate(idx):
            lo = off[t] + 8 * t
            hi = off[t + 1] + 8 * (t + 1)
            A0 = F["A"][F["ab_off"][i]:F["ab_off"][i + 1]]
            b0 = F["b"][F["ab_off"][i]:F["ab_off"][i + 1]]
            assert np.array_equal(A[lo:hi], A0), i
            assert np.array_equal(b[lo:hi], b0), i


def test_compat_get_safe_control(golden):
    """The reference's own call surface: ndarray (2,) out (cbf.py:92)."""
    F = golden("golden_filter.npz")
    c = cbf_amd.ControlBarrierFunction(15)
    fx = 0.1 * np.zeros((4, 4))
    for i in np.where(F["tag"] == 0)[0][:40]:
        obs = F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]]
        u = c.get_safe_control(F["r"][i], obs, fx, GX, F["u0"][i])
        assert isinstance(u, np.ndarray) and u.shape == (2,) and u.dtype == np.float64
        assert np.abs(u - F["u"][i]).max() <= 1e-12
    with pytest.raises(ValueError):
        c.get_safe_control(np.zeros(2), np.zeros((1, 2)), np.zeros((2, 2)), np.eye(2), [0.0, 0.0])


def test_compat_get_safe_control_sizes_and_threads():
    """get_safe_control's per-instance pinned buffers: no obstacle (m = 0), more than the initial
    64 obstacles (the buffers grow), and 8 threads sharing one instance (a lock keeps the call
    reentrant) -- every answer equal to the oracle's."""
    c = cbf_amd.ControlBarrierFunction(15)
    rng = np.random.default_rng(44)
    p = po.Params(15)
    cases = []
    for m in (0, 3, 65, 200, 1):
        r = np.concatenate([rng.uniform(-1, 1, 2), rng.normal(0, 0.3, 2)])
        obs = np.concatenate([r[:2] + rng.uniform(-0.3, 0.3, (m, 2)), rng.normal(0, 0.3, (m, 2))], axis=1)
        cases.append((r, obs, rng.normal(0, 1.0, 2)))
    want = [coracle.filter_one(p, r, obs, u0)["u"] for r, obs, u0 in cases]
    for (r, obs, u0), w in zip(cases, want):
        assert np.array_equal(c.get_safe_control(r, obs, np.zeros((4, 4)), GX, u0), w)

    def call(i):
        r, obs, u0 = cases[i % len(cases)]
        return i, c.get_safe_control(r, obs, np.zeros((4, 4)), GX, u0)
    with cf.ThreadPoolExecutor(8) as ex:
        for i, u in ex.map(call, range(80)):
            assert np.array_equal(u, want[i % len(cases)]), i


def _random_swarm(rng, n, n_obs, spread):
    pos = rng.uniform(-spread, spread, (n, 2))
    vel = rng.normal(0, 0.3, (n, 2))
    if n > 10:
        pos[3] = pos[5]                    # coincident
        pos[7] = pos[6] + [0.2, 0.0]       # exactly at the radius
        pos[8] = pos[9] + [np.nextafter(0.2, 0), 0.0]
        pos[10] = pos[6] + [-0.0, 0.1]     # dx = -0.0
    return pos, vel


@pytest.mark.parametrize("pset", paramsets.NAMES)
@pytest.mark.parametrize("method", ["allpairs", "cells"])
def test_filter_swarm_vs_oracle(method, pset):
    """cross_and_rescue.py:135-160 over random swarms, at the callers' parameters and at others
    (tests/paramsets.py: f != 0, random g, non-integer k, other dmin / max_speed / cull radius)."""
    rng = np.random.default_rng(11)
    p = paramsets.oracle_params(pset)
    fp = paramsets.filter_params(pset)
    for (n, n_obs, spread) in [(40, 10, 0.3), (700, 100, 1.5), (3000, 0, 2.5), (5000, 1500, 4.0)]:
        pos, vel = _random_swarm(rng, n, n_obs, spread)
        ref = coracle.filter_swarm(p, pos, vel, n_obs, kmax=64, diag=True)
        out = swarm.filter_swarm(fp, _t(pos), _t(vel), n_obs, method=method, kmax=64, diag=True)
        got = {k: v.cpu().numpy() for k, v in out.items()}
        assert np.array_equal(got["u"], ref["u"])
        assert np.array_equal(got["status"], ref["status"])
        assert np.array_equal(got["nbr_count"], ref["cnt"])
        assert np.array_equal(got["x"], ref["x"])
        assert np.array_equal(got["viol"], ref["viol"])
        assert np.array_equal(got["box_active"], ref["box_active"])
        for k in range(n - n_obs):
            m = min(ref["cnt"][k], 64)
            a = sorted(zip(got["nbr_idx"][k, :m].tolist(), got["nbr_active"][k, :m].tolist()))
            b = sorted(zip(ref["nbr_idx"][k, :m].tolist(), ref["nbr_active"][k, :m].tolist()))
            if method == "allpairs":
                assert a == list(zip(ref["nbr_idx"][k, :m].tolist(), ref["nbr_active"][k, :m].tolist()))
            if ref["cnt"][k] <= 64:
                assert a == b, (n, k)
        feas = np.isin(ref["status"] & 0xFF, [po.STATUS_OPTIMAL, po.STATUS_RELAXED])
        assert got["viol"][feas].max(initial=0.0) <= 1e-10   # feasibility tolerance 1e-12 max(1, |b|)


def test_consensus_vs_golden(golden):
    G = golden("golden_consensus.npz")
    for t in range(len(G["deg"])):
        deg = int(G["deg"][t])
        X = _t(G["X"][t][:, :deg + 1].T)
        rp = _t(np.array([0, deg], np.int32), torch.int32)
        col = _t(np.arange(1, deg + 1, dtype=np.int32), torch.int32)
        th = G["theta"][t]
        plain = swarm.consensus_csr(X, rp, col, 0).cpu().numpy()
        rot = swarm.consensus_csr(X, rp, col, 0, rot=(np.cos(th), np.sin(th)), scale=G["scale"][t]).cpu().numpy()
        assert np.array_equal(plain[0], G["plain"][t])
        assert np.array_equal(rot[0], G["rot"][t])


def test_lattice_consensus_and_euler_vs_oracle():
    W, H = 37, 23
    pos = scenarios.lattice(W, H, seed=3)
    out = swarm.consensus_lattice(_t(pos), W, H, 0.25).cpu().numpy()
    assert np.array_equal(out, coracle.consensus_lattice(W, H, 0, H, pos, 0.25))
    part = swarm.consensus_lattice(_t(pos[5 * W:15 * W]), W, H, 0.25, row_begin=6, row_end=14,
                                   pos_row0=5).cpu().numpy()
    assert np.array_equal(part, coracle.consensus_lattice(W, H, 6, 14, pos, 0.25))
    vel = np.random.default_rng(0).normal(0, 1, pos.shape)
    p = _t(pos)
    swarm.euler(p, _t(vel), 1 / 30)
    assert np.array_equal(p.cpu().numpy(), coracle.euler(pos, vel, 1 / 30))


@pytest.mark.parametrize("name", ["cross_and_rescue", "meet_at_center", "meet_at_center_n100"])
def test_group_swarm_steps_vs_golden(golden, name):
    """One GPU step from each recorded state of the restated caller loops."""
    R = golden(f"golden_{name}.npz")
    if name == "cross_and_rescue":
        pos0, n_obs, groups = scenarios.cross_and_rescue()
    else:
        pos0, n_obs, groups = scenarios.meet_at_center(10 if name == "meet_at_center" else 100)
    assert np.array_equal(pos0, R["pos"][0])       # restated initial conditions
    S = swarm.GroupSwarm(pos0, n_obs, groups)
    for t in range(R["pos"].shape[0]):
        S.pos.copy_(_t(R["pos"][t]))
        out = S.step(kmax=S.n)
        assert np.array_equal(out["nominal"].cpu().numpy(), R["vel"][t]), t
        cnt = out["nbr_count"].cpu().numpy(); idx = out["nbr_idx"].cpu().numpy()
        for k in range(S.n - n_obs):
            assert set(idx[k, :cnt[k]].tolist()) == set(np.where(R["nbr_mask"][t][k])[0].tolist()), (t, k)
        u = out["u_all"].cpu().numpy()
        ref_u = R["u"][t] if R["u"][t].shape[0] == S.n else np.concatenate([R["vel"][t][:n_obs], R["u"][t]])
        assert np.abs(u - ref_u).max() <= 1e-12, t
        its = np.where(cnt > 0, out["status"].cpu().numpy() >> 8, 0)
        assert np.array_equal(its, R["relax_iters"][t]), t


def _oracle_group_rollout(pos, n_obs, groups, steps, T=1 / 30):
    p = po.Params(15)
    pos = pos.copy()
    for _ in range(steps):
        vel = np.zeros_like(pos)
        for (b, e, rows, anc, rot, scale) in groups:
            rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
            col = np.array([j for r in rows for j in r], np.int32)
            vel[b:e] = coracle.consensus_csr(pos[b:e], rp, col, 0, e - b, anchors=anc, rot=rot, scale=scale)
        out = coracle.filter_swarm(p, pos, vel, n_obs)
        u = vel.copy(); u[n_obs:] = out["u"]
        pos = coracle.euler(pos, u, T)
    return pos


@pytest.mark.parametrize("cfg", ["car", "mac10", "mac100"])
def test_group_swarm_rollout_bit_exact(cfg):
    """Multi-step GPU rollout == oracle rollout bit for bit (cfg1 / cfg2)."""
    if cfg == "car":
        pos0, n_obs, groups = scenarios.cross_and_rescue(); steps = 300
    elif cfg == "mac10":
        pos0, n_obs, groups = scenarios.meet_at_center(10); steps = 300
    else:
        pos0, n_obs, groups = scenarios.meet_at_center(100); steps = 100
    S = swarm.GroupSwarm(pos0, n_obs, groups)
    for _ in range(steps):
        S.step()
    ref = _oracle_group_rollout(pos0, n_obs, groups, steps)
    assert np.array_equal(S.pos.cpu().numpy(), ref)


def _oracle_lattice_step(pos, W, H, gain, T):
    vel = coracle.consensus_lattice(W, H, 0, H, pos, gain)
    out = coracle.filter_swarm(po.Params(15), pos, vel, 0)
    return coracle.euler(pos, out["u"], T), vel, out


def _oracle_stats(outs):
    """The rollout statistics (include/cbf_amd.h CBF_STAT_*) restated from oracle outputs."""
    st = {"solves": 0, "optimal": 0, "relaxed": 0, "infeasible": 0, "viol_optimal": 0.0,
          "viol_original_relaxed": 0.0, "min_dist2": np.inf, "binding": 0}
    for o in outs:
        code = o["status"] & 0xFF
        solved = o["cnt"] > 0
        st["solves"] += int(solved.sum())
        st["optimal"] += int((code == 1).sum())
        st["relaxed"] += int((code == 2).sum())
        st["infeasible"] += int(((code == 3) | (code == 4)).sum())
        st["viol_optimal"] = max(st["viol_optimal"], float(o["viol"][code == 1].max(initial=0.0)))
        st["viol_original_relaxed"] = max(st["viol_original_relaxed"],
                                          float(o["viol_orig"][code == 2].max(initial=0.0)))
        st["min_dist2"] = min(st["min_dist2"], float(o["d2min"].min(initial=np.inf)))
        st["binding"] += int((solved & (np.abs(o["x"]).max(axis=1) > 0)).sum())
    return st


def _check_stats(got, want):
    for k in ("solves", "optimal", "relaxed", "infeasible", "binding", "viol_optimal", "viol_original_relaxed"):
        assert got[k] == want[k], (k, got[k], want[k])
    assert (got["min_dist2"] if got["min_dist2"] is not None else np.inf) == want["min_dist2"]
    assert got["seidel"] <= got["binding"] + got["relaxed"] + got["infeasible"]
    assert got["errors"] == 0


# Both placements of the full QP solve (cbf_params.solve_inline_max): inline in the filter (what
# the shipped library picks for windows of <= 131072 agents) and queued for k_lattice_filter_hard
# (its pick above that: the path the 1 M-agent bench times).  Every lattice test against the oracle
# runs both, so each is anchored to the oracle on its own.
PLACEMENTS = ["inline", "queued"]
# ... and both culls of the lattice step: the cell list, and the lattice-window cull
# (CBF_RUN_WINDOW_CULL: lattice neighbours as candidates, guards proving the rest out of range)
VARIANTS = [(pl, cull) for cull in ("cells", "window") for pl in PLACEMENTS]


def _fp(placement, pset="callers"):
    return paramsets.filter_params(pset, solve_placement=placement)


def _kw(variant, pset="callers"):
    placement, cull = variant
    return {"params": _fp(placement, pset), "cull": cull}


@pytest.mark.parametrize("pset", paramsets.NAMES)
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("spacing", [scenarios.LATTICE_SPACING, 0.2])
def test_lattice_step_vs_oracle(spacing, variant, pset):
    """Fused lattice steps == oracle steps bit for bit, and the device rollout statistics (status
    counts, OPTIMAL-only and original-row violations, minimum neighbour distance) equal the same
    quantities restated from the oracle's outputs.  Spacing 0.2 is the feasible regime (cfg4f).
    pset: the callers' parameters, or others (tests/paramsets.py) -- the f != 0 instantiations,
    and with the 0.3 cull radius the window cull's walk beyond its staged tile."""
    W, H = 48, 40
    pos = scenarios.lattice(W, H, seed=5, spacing=spacing)
    L = swarm.LatticeSwarm(pos, W, H, gain=0.25, **_kw(variant, pset))
    p = paramsets.oracle_params(pset)
    ref = pos.copy()
    outs = []
    for step in range(8):
        L.step()
        vel = coracle.consensus_lattice(W, H, 0, H, ref, 0.25)
        out = coracle.filter_swarm(p, ref, vel, 0, diag=True, stats=True)
        ref = coracle.euler(ref, out["u"], 1 / 30)
        outs.append(out)
        assert np.array_equal(L.vel.cpu().numpy(), vel), step
        assert np.array_equal(L.u.cpu().numpy(), out["u"]), step
        assert np.array_equal(L.status.cpu().numpy(), out["status"]), step
        assert np.array_equal(L.nbr_count.cpu().numpy(), out["cnt"]), step
        assert np.array_equal(L.pos.cpu().numpy(), ref), step
    want = _oracle_stats(outs)
    _check_stats(L.stats_summary(), want)
    if spacing == 0.2 and pset == "callers":
        assert want["optimal"] > 0.5 * want["solves"] and want["binding"] > 0.1 * want["solves"]


@pytest.mark.parametrize("pset", ["callers", "nondefault"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_lattice_random_nominal_vs_oracle(variant, pset):
    """The random-walk nominal control (CBF_NOMINAL_RANDOM, the exact-QP regime cfg4r): fused
    steps == oracle steps bit for bit (nominal controls, controls, statuses, positions, rollout
    statistics); most QPs are feasible with a binding row; cbf_lattice_run (chained binning) and
    a hipGraph of run(4) give the same rollout."""
    W, H, amp, seed = 48, 40, 1.0, 3
    pos = scenarios.lattice(W, H, seed=5, spacing=0.22)
    kw = _kw(variant, pset)
    p = paramsets.oracle_params(pset)
    L = swarm.LatticeSwarm(pos, W, H, nominal=("random", amp, seed), **kw)
    ref = pos.copy()
    outs = []
    for step in range(8):
        L.step()
        vel = po.random_nominal(ref, 0, amp, seed)
        out = coracle.filter_swarm(p, ref, vel, 0, diag=True, stats=True)
        ref = coracle.euler(ref, out["u"], 1 / 30)
        outs.append(out)
        assert np.array_equal(L.vel.cpu().numpy(), vel), step
        assert np.array_equal(L.u.cpu().numpy(), out["u"]), step
        assert np.array_equal(L.status.cpu().numpy(), out["status"]), step
        assert np.array_equal(L.pos.cpu().numpy(), ref), step
    want = _oracle_stats(outs)
    _check_stats(L.stats_summary(), want)
    if pset == "callers":
        assert want["optimal"] > 0.6 * want["solves"] and want["binding"] > 0.4 * want["solves"]
    B = swarm.LatticeSwarm(pos, W, H, nominal=("random", amp, seed), **kw)
    B.run(3)
    B.run(5)
    for a, b in zip(_lattice_state(L), _lattice_state(B)):
        assert np.array_equal(a, b)
    D = swarm.LatticeSwarm(pos, W, H, nominal=("random", amp, seed), **kw)
    D.capture(steps=4)              # the capture's warm-up launch runs steps 1-4
    D.run(4)
    for a, b in zip(_lattice_state(L), _lattice_state(D)):
        assert np.array_equal(a, b)


def test_lattice_graph_replay_matches_eager():
    W, H = 64, 64
    pos = scenarios.lattice(W, H, seed=9)
    A = swarm.LatticeSwarm(pos, W, H)
    B = swarm.LatticeSwarm(pos, W, H)
    B.capture()
    torch.cuda.synchronize()
    B.pos.copy_(_t(pos))          # capture ran one warm-up step; restart from pos
    for _ in range(5):
        A.step()
        B.step()
    torch.cuda.synchronize()
    assert torch.equal(A.pos, B.pos) and torch.equal(A.u, B.u)


def _lattice_state(L):
    """Positions, last-step outputs, and the decoded statistics (the raw words are per-slot
    partial sums whose split over the slots follows queue order)."""
    torch.cuda.synchronize()
    st = L.stats_summary()
    return [t.cpu().numpy().copy() for t in (L.pos, L.vel, L.u, L.status, L.nbr_count)] + \
        [np.array([st[k] for k in sorted(st)], dtype=object)]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("spacing", [scenarios.LATTICE_SPACING, 0.2])
def test_lattice_run_matches_steps(spacing, variant):
    """cbf_lattice_run (chained binning: each advance bins the next timestep) == the same number of
    cbf_lattice_step calls, bit for bit: positions, last-step outputs and every statistics word,
    in one call, split over calls, and replayed from a hipGraph of run(4).  The first 3 steps of
    the reference run are also checked against the oracle, so the chain is anchored to it.  With
    the queued placement the chained binning of the queued egos runs in the queue kernel."""
    W, H = 256, 192
    pos = scenarios.lattice(W, H, seed=11, spacing=spacing)
    kw = _kw(variant)
    A = swarm.LatticeSwarm(pos, W, H, **kw)
    ref = pos.copy()
    states = {}
    for k in range(1, 17):
        A.step()
        if k <= 3:
            vel = coracle.consensus_lattice(W, H, 0, H, ref, 0.25)
            ref = coracle.euler(ref, coracle.filter_swarm(po.Params(15), ref, vel, 0)["u"], 1 / 30)
            assert np.array_equal(A.pos.cpu().numpy(), ref), k
        if k in (12, 16):
            states[k] = _lattice_state(A)
    B = swarm.LatticeSwarm(pos, W, H, **kw)
    B.run(12)
    for a, b in zip(states[12], _lattice_state(B)):
        assert np.array_equal(a, b)
    C = swarm.LatticeSwarm(pos, W, H, **kw)
    for n in (1, 5, 6):
        C.run(n)
    for a, b in zip(states[12], _lattice_state(C)):
        assert np.array_equal(a, b)
    D = swarm.LatticeSwarm(pos, W, H, **kw)
    D.capture(steps=4)              # the capture's warm-up launch runs steps 1-4
    for _ in range(3):
        D.run(4)
    for a, b in zip(states[16], _lattice_state(D)):
        assert np.array_equal(a, b)
    st = B.stats_summary()
    assert st["errors"] == 0 and st["solves"] > 0
    if spacing == 0.2:
        # full solves happen; queued, the queue kernel bins them for the next timestep (the chained
        # binning of k_lattice_filter_hard), inline the filter does
        assert st["seidel"] > 0


def test_lattice_run_output_history():
    """cbf_lattice_run_ex(CBF_RUN_OUTPUT_HISTORY): every timestep's nominal control, filtered
    control, status and neighbour count (the reference's per-step si_velocities) equal those of
    the corresponding step() call, and the trajectory is the plain run's, bit for bit; also from a
    hipGraph of run(5, history=True)."""
    W, H = 160, 128
    pos = scenarios.lattice(W, H, seed=12, spacing=0.2)
    A = swarm.LatticeSwarm(pos, W, H)
    per_step = []
    for _ in range(10):
        A.step()
        per_step.append((A.vel.clone(), A.u.clone(), A.status.clone(), A.nbr_count.clone()))
    B = swarm.LatticeSwarm(pos, W, H)
    B.run(5, history=True)
    hist = [t.clone() for t in B.history(5)]
    B.capture(steps=5, history=True)   # the capture's warm-up launch runs timesteps 6-10
    torch.cuda.synchronize()
    hist2 = B.history(5)
    for t in range(10):
        got = [h[t] for h in hist] if t < 5 else [h[t - 5] for h in hist2]
        for a, b in zip(per_step[t], got):
            assert torch.equal(a, b), t
    assert torch.equal(A.pos, B.pos)
    B.run(5, history=True)            # graph replay: timesteps 11-15
    C = swarm.LatticeSwarm(pos, W, H)
    C.run(15)
    torch.cuda.synchronize()
    assert torch.equal(C.pos, B.pos) and torch.equal(C.u, B.history(5)[1][4])


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("nominal", [None, ("random", 0.05, 3)])
def test_lattice_stats_off_and_replay(nominal, variant):
    """The bench's timed path: run() with stats=NULL (graphs of both modes captured) gives the same
    trajectory bit for bit as with the statistics on, and snapshot()/restore() makes the statistics
    replay repeat a stats-off rollout exactly (positions, outputs), with the replay's statistics
    equal to those of a stats-on rollout from the start (incl. the random-walk nominal state)."""
    W, H = 128, 96
    pos = scenarios.lattice(W, H, seed=5, spacing=0.2)
    A = swarm.LatticeSwarm(pos, W, H, nominal=nominal, **_kw(variant))
    A.run(6)
    B = swarm.LatticeSwarm(pos, W, H, nominal=nominal, **_kw(variant))
    B.collect_stats = False
    B.capture(steps=3)              # runs steps 1-3 (stats off)
    B.collect_stats = True
    B.capture(steps=3)              # runs steps 4-6 (stats on)
    B.reset_solves()
    torch.cuda.synchronize()
    assert torch.equal(A.pos, B.pos) and torch.equal(A.u, B.u) and torch.equal(A.status, B.status)
    snap = B.snapshot()
    ref = swarm.LatticeSwarm(pos, W, H, nominal=nominal, **_kw(variant))
    ref.run(6)
    ref.reset_solves()
    ref.run(8)                      # the statistics of steps 7-14 alone
    B.collect_stats = False
    for _ in range(2):
        B.run(3)
    B.run(2)
    torch.cuda.synchronize()
    end = [t.clone() for t in (B.pos, B.u, B.status)]
    assert int(B.stats.abs().sum()) == 0   # nothing recorded with stats=NULL
    B.restore(snap)
    B.collect_stats = True
    B.reset_solves()
    for _ in range(2):
        B.run(3)
    B.run(2)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(end, (B.pos, B.u, B.status)))
    assert torch.equal(B.pos, ref.pos)
    sa, sb = ref.stats_summary(), B.stats_summary()
    assert sa == sb and sb["solves"] > 0 and sb["errors"] == 0


def test_lattice_advance_marked_equals_advance():
    """cbf_lattice_advance_marked (the bench's measurement hook) == cbf_lattice_advance bit for bit,
    and its event lands between the start and the end of the advance call."""
    W, H = 96, 64
    pos = scenarios.lattice(W, H, seed=8, spacing=0.2)
    A = swarm.LatticeSwarm(pos, W, H)
    B = swarm.LatticeSwarm(pos, W, H)
    A.build_phase()
    A.advance_phase()
    B.build_phase()
    a, m, b = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    m.record()
    a.record()
    B.advance_phase(mark=m)
    b.record()
    torch.cuda.synchronize()
    assert torch.equal(A.pos, B.pos) and torch.equal(A.u, B.u) and torch.equal(A.status, B.status)
    assert 0 <= a.elapsed_time(m) <= a.elapsed_time(b)


def _sample_oracle(pos, vel, idx, threads=16):
    p = po.Params(15)
    chunks = np.array_split(idx, threads)

    def run(ch):
        res = []
        for e in ch:
            o = coracle.filter_swarm(p, pos, vel, 0, int(e), int(e) + 1)
            res.append((o["u"][0], o["status"][0], o["cnt"][0]))
        return res
    with cf.ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(run, chunks))
    return [r for part in parts for r in part]


def test_lattice_full_size_cfg4():
    """cfg4 at full size (1024 x 1024): a sample of egos checked against the O(N) reference cull
    of the oracle, plus size-independent properties over all agents."""
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0)
    L = swarm.LatticeSwarm(pos, W, H)
    L.step()
    torch.cuda.synchronize()
    vel = L.vel.cpu().numpy()
    assert np.array_equal(vel, coracle.consensus_lattice(W, H, 0, H, pos, 0.25))
    u, st, cnt = L.u.cpu().numpy(), L.status.cpu().numpy(), L.nbr_count.cpu().numpy()
    idx = np.random.default_rng(1).choice(W * H, 256, replace=False)
    for e, (ru, rst, rc) in zip(idx, _sample_oracle(pos, vel, idx)):
        assert np.array_equal(u[e], ru) and st[e] == rst and cnt[e] == rc, e
    # properties: Euler consistency, status domain, idle => u0 passthrough, |u| <= ms when filtered
    assert np.array_equal(L.pos.cpu().numpy(), coracle.euler(pos, u, 1 / 30))
    code = st & 0xFF
    assert set(np.unique(code)).issubset({0, 1, 2, 3, 4})
    assert np.array_equal(code == 0, cnt == 0)
    assert np.array_equal(u[cnt == 0], vel[cnt == 0])
    assert np.abs(u[cnt > 0]).max() <= 15.0


def _min_pair_dist2(pos, cull_t):
    """Exact smallest s = dx^2 + dy^2 over pairs with 0 < s < cull_t (the GPU's and the oracle's
    arithmetic: the pair's two egos compute the same s, negation being exact)."""
    from scipy.spatial import cKDTree
    pr = cKDTree(pos).query_pairs(0.2 * (1 + 1e-9), output_type="ndarray")
    d = pos[pr[:, 1]] - pos[pr[:, 0]]
    s = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]
    s = s[(s < cull_t) & (s > 0)]
    return float(s.min()) if s.size else np.inf


@pytest.mark.parametrize("spacing", [scenarios.LATTICE_SPACING, 0.2])
def test_lattice_full_size_safety_stats(spacing):
    """cfg4 (and the feasible-regime cfg4f) at full size, 1024 x 1024, over a 3-step rollout: the
    OPTIMAL-only row violation is <= 1e-12 (north star <= 1e-7), the device statistics count every
    agent-QP once and agree with the statuses, and the minimum neighbour distance equals the exact
    minimum over all culled pairs of the steps' input states."""
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0, spacing=spacing)
    L = swarm.LatticeSwarm(pos, W, H)
    cull_t = float(swarm.FilterParams().c().cull_t)
    d2 = []
    codes = np.zeros(8, np.int64)
    for _ in range(3):
        d2.append(_min_pair_dist2(L.pos.cpu().numpy(), cull_t))
        L.step()
        st = L.status.cpu().numpy() & 0xFF
        codes += np.bincount(st, minlength=8)
    got = L.stats_summary()
    assert got["errors"] == 0
    assert got["solves"] == codes[1] + codes[2] + codes[3] + codes[4]
    assert (got["optimal"], got["relaxed"], got["infeasible"]) == (codes[1], codes[2], codes[3] + codes[4])
    assert got["viol_optimal"] <= 1e-12
    assert got["min_dist2"] == min(d2)
    if spacing == 0.2:   # the feasible regime: most QPs feasible, rows binding for many
        assert got["optimal"] > 0.6 * got["solves"] and got["binding"] > 0.15 * got["solves"]
    else:
        assert got["relaxed"] > 0.9 * got["solves"] and got["viol_original_relaxed"] > 0


def test_lattice_full_size_cfg3_allpairs():
    """cfg3 at full size (256 x 256 = 65,536 agents, every pair tested): one step, 256 sampled egos
    against the O(N) reference cull of the oracle, plus size-independent properties."""
    W = H = 256
    pos = scenarios.lattice(W, H, seed=0)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, method="allpairs")
    L.step()
    torch.cuda.synchronize()
    vel = coracle.consensus_lattice(W, H, 0, H, pos, scenarios.LATTICE_GAIN)
    assert np.array_equal(L.vel.cpu().numpy(), vel)
    u, st, cnt = L.u.cpu().numpy(), L.status.cpu().numpy(), L.nbr_count.cpu().numpy()
    idx = np.random.default_rng(3).choice(W * H, 256, replace=False)
    for e, (ru, rst, rc) in zip(idx, _sample_oracle(pos, vel, idx)):
        assert np.array_equal(u[e], ru) and st[e] == rst and cnt[e] == rc, e
    assert np.array_equal(L.pos.cpu().numpy(), coracle.euler(pos, u, 1 / 30))
    code = st & 0xFF
    assert np.array_equal(code == 0, cnt == 0)
    assert np.array_equal(u[cnt == 0], vel[cnt == 0])
    # the cell-list filter (a different cull) agrees on the whole swarm
    out = swarm.filter_swarm(swarm.FilterParams(), _t(pos), _t(vel), 0, method="cells")
    assert np.array_equal(out["u"].cpu().numpy(), u) and np.array_equal(out["status"].cpu().numpy(), st)


@pytest.mark.parametrize("pset", paramsets.NAMES)
def test_mc_rollout_vs_oracle(pset):
    p = paramsets.oracle_params(pset)
    n_scen, n_o, n_a, steps = 40, 16, 16, 60
    pos0 = scenarios.mc_scenarios(n_scen, n_o, n_a, seed=4)
    P = _t(pos0)
    cnt, mv, sf = swarm.mc_rollout(paramsets.filter_params(pset), P, n_o, n_a, steps, ga=scenarios.MC_GAIN,
                                   safety=True)
    rp, rc, rm, rs = coracle.mc_rollout(p, pos0, n_o, n_a, steps, 1 / 30,
                                        (np.cos(-np.pi / n_o), np.sin(-np.pi / n_o)), 1.0, scenarios.MC_GAIN,
                                        safety=True)
    assert np.array_equal(P.cpu().numpy(), rp)
    assert np.array_equal(cnt.cpu().numpy(), rc)
    assert np.array_equal(mv.cpu().numpy(), rm)
    assert np.array_equal(sf.cpu().numpy(), rs)
    assert rc[:, 0].sum() > 0 and rm.max() <= 1e-10   # feasibility tolerance 1e-12 max(1, |b|)


def test_mc_rollout_full_batch_cfg5():
    """cfg5 at full size: 100,000 scenarios x 32 entities, 10 steps in one launch; 64 sampled
    scenarios checked bit for bit against the oracle's rollout (positions, counters, violations,
    distances), and the whole batch's OPTIMAL-only violation <= 1e-12."""
    p = po.Params(15)
    n_scen, n_o, n_a, steps = 100_000, 16, 16, 10
    pos0 = scenarios.mc_scenarios(n_scen, n_o, n_a, seed=0)
    P = _t(pos0)
    cnt, mv, sf = swarm.mc_rollout(swarm.FilterParams(), P, n_o, n_a, steps, ga=scenarios.MC_GAIN, safety=True)
    got_p, got_c, got_m, got_s = P.cpu().numpy(), cnt.cpu().numpy(), mv.cpu().numpy(), sf.cpu().numpy()
    idx = np.sort(np.random.default_rng(5).choice(n_scen, 64, replace=False))
    rp, rc, rm, rs = coracle.mc_rollout(p, pos0[idx], n_o, n_a, steps, 1 / 30,
                                        (np.cos(-np.pi / n_o), np.sin(-np.pi / n_o)), 1.0, scenarios.MC_GAIN,
                                        safety=True)
    assert np.array_equal(got_p[idx], rp)
    assert np.array_equal(got_c[idx], rc)
    assert np.array_equal(got_m[idx], rm)
    assert np.array_equal(got_s[idx], rs)
    assert got_c[:, 0].sum() > 0 and got_m.max() <= 1e-12
    assert np.isfinite(got_p).all()


def test_mc_rollout_shipped_meet_at_center_shape():
    """n_o = n_a = 5 (meet_at_center.py) and an odd mix, bit-exact vs oracle."""
    p = po.Params(15)
    for (n_o, n_a) in [(5, 5), (7, 12)]:
        pos0 = scenarios.mc_scenarios(33, n_o, n_a, seed=n_o)
        P = _t(pos0)
        cnt, mv = swarm.mc_rollout(swarm.FilterParams(), P, n_o, n_a, 40, ga=1.0)
        rp, rc, rm = coracle.mc_rollout(p, pos0, n_o, n_a, 40, 1 / 30,
                                        (np.cos(-np.pi / n_o), np.sin(-np.pi / n_o)), 1.0, 1.0)
        assert np.array_equal(P.cpu().numpy(), rp)
        assert np.array_equal(cnt.cpu().numpy(), rc)


def test_invalid_arguments_raise():
    fp = swarm.FilterParams()
    pos = _t(np.zeros((4, 2)))
    with pytest.raises(cbf_amd.CbfError):
        swarm.filter_swarm(fp, pos, pos, 5)   # n_obs > n
    bad = swarm.make_grid(0, 0, 1, 1, 0.1)   # cell edge smaller than the cull radius
    with pytest.raises(cbf_amd.CbfError):
        swarm.filter_swarm(fp, pos, pos, 0, method="cells", grid=bad)


def test_gpu_vs_restated_cvxopt_feasible(golden):
    """North-star gate "controls within 1e-5 of cvxopt", against the restatement of cvxopt's coneqp
    (oracle/cvxqp.py; the binary is absent, so parity vs cvxopt itself stays unpinned): every
    feasible golden QP within the IPM's own certified distance sqrt(2 gap), >= 98 % within 1e-5."""
    from oracle import cvxqp
    F = golden("golden_filter.npz")
    errs = []
    for (ms, dmin, k, gb, fb), idx in _golden_groups(F).items():
        g = np.frombuffer(gb, dtype=np.float64).reshape(4, 2)
        f = np.frombuffer(fb, dtype=np.float64).reshape(4, 4)
        c = cbf_amd.ControlBarrierFunction(ms, dmin=dmin, k=k)
        obs = [F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]] for i in idx]
        off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int32)
        u, st, x = c.get_safe_control_batch(_t(F["r"][idx]), (_t(off, torch.int32), _t(np.vstack(obs))),
                                            _t(F["u0"][idx]), f=f, g=g, return_x=True)
        u, x = u.cpu().numpy(), x.cpu().numpy()
        for t, i in enumerate(idx):
            if int(F["relax_iters"][i]) != 0:
                continue
            A = F["A"][F["ab_off"][i]:F["ab_off"][i + 1]]
            b = F["b"][F["ab_off"][i]:F["ab_off"][i + 1]]
            uc, sol = cvxqp.get_safe_control(A, b, len(b) - 8, F["u0"][i], ms)
            assert sol["status"] == "optimal", i
            assert np.linalg.norm(x[t] - sol["x"]) <= np.sqrt(2 * max(sol["gap"], 0.0)) + 1e-9, i
            errs.append(float(np.abs(u[t] - uc).max()))
    errs = np.array(errs)
    assert len(errs) > 700 and (errs <= 1e-5).mean() >= 0.98


@pytest.mark.parametrize("offset", [0.0, 1e3, 1e6, 1e12, 1e31])
def test_allpairs_screen_exact_at_any_magnitude(offset):
    """The all-pairs kernel's fp32 screen only rejects candidates that the exact fp64 test rejects:
    neighbour sets and controls stay bit-identical to the oracle with coordinates far from the
    origin (coarse fp32 rounding, wider screen margin) and beyond 1e30 (screen switched off)."""
    rng = np.random.default_rng(5)
    p = po.Params(15)
    fp = swarm.FilterParams()
    n, n_obs = 600, 60
    pos, vel = _random_swarm(rng, n, n_obs, 1.0)
    # pairs straddling the cull radius (s just below / at / above cull_t)
    for i, d in enumerate([np.nextafter(0.2, 0), 0.2, np.nextafter(0.2, 1), 0.19999999, 0.20000001]):
        pos[100 + 2 * i + 1] = pos[100 + 2 * i] + [d, 0.0]
        pos[200 + 2 * i + 1] = pos[200 + 2 * i] + [d * 0.6, d * 0.8]
    pos = pos + offset
    ref = coracle.filter_swarm(p, pos, vel, n_obs, kmax=32, diag=True)
    out = swarm.filter_swarm(fp, _t(pos), _t(vel), n_obs, method="allpairs", kmax=32, diag=True)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert np.array_equal(got["nbr_count"], ref["cnt"])
    assert np.array_equal(got["nbr_idx"], ref["nbr_idx"])
    assert np.array_equal(got["u"], ref["u"])
    assert np.array_equal(got["status"], ref["status"])


def test_allpairs_nonfinite_coordinates():
    rng = np.random.default_rng(6)
    p = po.Params(15)
    fp = swarm.FilterParams()
    pos, vel = _random_swarm(rng, 300, 30, 0.8)
    pos[40] = [np.nan, 0.1]
    pos[41] = [np.inf, 0.0]
    pos[290] = [0.05, np.nan]
    ref = coracle.filter_swarm(p, pos, vel, 30, kmax=32, diag=True)
    out = swarm.filter_swarm(fp, _t(pos), _t(vel), 30, method="allpairs", kmax=32, diag=True)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert np.array_equal(got["nbr_count"], ref["cnt"])
    assert np.array_equal(got["nbr_idx"], ref["nbr_idx"])
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["u"], ref["u"], equal_nan=True)


@pytest.mark.parametrize("offset", [0.0, 37.0, 150.0, 260.0, 1e3, 1e31])
def test_allpairs_split_screen_exact_at_any_magnitude(offset):
    """Split all-pairs (scalar-operand screen): the expanded-form fp32 screen (used while
    16 u M^2 <= cull_t, M <~ 200), the difference form beyond it, and no screen beyond 1e30 all
    only reject what the exact test rejects.  Pairs straddle the cull radius; a few entities sit
    at large magnitude so that some waves mix the two forms."""
    rng = np.random.default_rng(15)
    p = po.Params(15)
    fp = swarm.FilterParams()
    n, n_obs = 2000, 100
    pos, vel = _random_swarm(rng, n, n_obs, 2.0)
    for i, d in enumerate([np.nextafter(0.2, 0), 0.2, np.nextafter(0.2, 1), 0.19999999, 0.20000001]):
        pos[300 + 2 * i + 1] = pos[300 + 2 * i] + [d, 0.0]
        pos[500 + 2 * i + 1] = pos[500 + 2 * i] + [d * 0.6, d * 0.8]
        pos[700 + 2 * i + 1] = pos[700 + 2 * i] + [-d * 0.8, d * 0.6]
    pos = pos + offset
    pos[1500:1510] += 5e3  # a wave whose egos need the difference form, next to expanded ones
    pos[1510:1512] = pos[1500:1502] + [0.1, 0.1]
    ref = coracle.filter_swarm(p, pos, vel, n_obs)
    out = swarm.filter_swarm(fp, _t(pos), _t(vel), n_obs, method="allpairs")
    assert np.array_equal(out["nbr_count"].cpu().numpy(), ref["cnt"])
    assert np.array_equal(out["u"].cpu().numpy(), ref["u"])
    assert np.array_equal(out["status"].cpu().numpy(), ref["status"])


def test_allpairs_split_nonfinite_coordinates():
    rng = np.random.default_rng(16)
    p = po.Params(15)
    fp = swarm.FilterParams()
    pos, vel = _random_swarm(rng, 700, 30, 0.8)
    pos[40] = [np.nan, 0.1]
    pos[41] = [np.inf, 0.0]
    pos[690] = [0.05, np.nan]
    ref = coracle.filter_swarm(p, pos, vel, 30)
    out = swarm.filter_swarm(fp, _t(pos), _t(vel), 30, method="allpairs")
    assert np.array_equal(out["nbr_count"].cpu().numpy(), ref["cnt"])
    assert np.array_equal(out["status"].cpu().numpy(), ref["status"])
    assert np.array_equal(out["u"].cpu().numpy(), ref["u"], equal_nan=True)


@pytest.mark.parametrize("n,n_obs,spread", [(40, 10, 0.3), (5000, 1500, 4.0), (20000, 0, 6.0)])
def test_allpairs_split_vs_oracle(n, n_obs, spread):
    """cbf_filter_allpairs_split (candidate chunks in separate workgroups, merged in order) gives
    the same controls, statuses and neighbour counts as the oracle's sequential loop."""
    rng = np.random.default_rng(n)
    p = po.Params(15)
    fp = swarm.FilterParams()
    pos, vel = _random_swarm(rng, n, n_obs, spread)
    ref = coracle.filter_swarm(p, pos, vel, n_obs)
    out = swarm.filter_swarm(fp, _t(pos), _t(vel), n_obs, method="allpairs")
    assert np.array_equal(out["u"].cpu().numpy(), ref["u"])
    assert np.array_equal(out["status"].cpu().numpy(), ref["status"])
    assert np.array_equal(out["nbr_count"].cpu().numpy(), ref["cnt"])


def test_lattice_allpairs_step_vs_oracle():
    """cfg3 shape (every pair tested) at 64 x 64: consensus + split all-pairs filter + Euler."""
    W = H = 64
    pos = scenarios.lattice(W, H, seed=3)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, method="allpairs")
    L.step()
    torch.cuda.synchronize()
    vel = coracle.consensus_lattice(W, H, 0, H, pos, scenarios.LATTICE_GAIN)
    ref = coracle.filter_swarm(po.Params(15), pos, vel, 0)
    assert np.array_equal(L.u.cpu().numpy(), ref["u"])
    assert np.array_equal(L.pos.cpu().numpy(), coracle.euler(pos, ref["u"], 1 / 30))


def test_workspace_bound_to_its_shape():
    """A cells workspace reused with another grid is refused on the device (every ego reports
    CBF_STATUS_WORKSPACE_ERROR, unfiltered) until it is zero-filled again (include/cbf_amd.h)."""
    rng = np.random.default_rng(21)
    p = po.Params(15)
    fp = swarm.FilterParams()
    pos, vel = _random_swarm(rng, 3000, 0, 2.5)
    ref = coracle.filter_swarm(p, pos, vel, 0)
    g1 = swarm.grid_for_points(pos, 0.2)
    g2 = swarm.grid_for_points(pos, 0.2, margin=3.0)
    from cbf_amd import _lib
    need = max(_lib.lib.cbf_cells_workspace_size(3000, _lib.C.byref(g)) for g in (g1, g2))
    ws = torch.zeros((need,), dtype=torch.uint8, device=DEV)
    a = swarm.filter_swarm(fp, _t(pos), _t(vel), 0, method="cells", grid=g1, workspace=ws)
    assert np.array_equal(a["u"].cpu().numpy(), ref["u"])
    b = swarm.filter_swarm(fp, _t(pos), _t(vel), 0, method="cells", grid=g1, workspace=ws)   # same shape: fine
    assert np.array_equal(b["status"].cpu().numpy(), ref["status"])
    for _ in range(2):   # another grid: refused, and stays refused
        c = swarm.filter_swarm(fp, _t(pos), _t(vel), 0, method="cells", grid=g2, workspace=ws)
        assert (c["status"].cpu().numpy() == _lib.STATUS_WORKSPACE_ERROR).all()
        assert np.array_equal(c["u"].cpu().numpy(), vel)
    ws.zero_()
    d = swarm.filter_swarm(fp, _t(pos), _t(vel), 0, method="cells", grid=g2, workspace=ws)
    assert np.array_equal(d["u"].cpu().numpy(), ref["u"])


def test_scan_timeout_is_reported():
    """A scan look-back that gives up (forced in every tile by the test-only build
    tests/_lib/libcbf_scantimeout.so, CBF_SCAN_TEST_TIMEOUT) is reported, not silent: every ego of
    the step gets CBF_STATUS_WORKSPACE_ERROR and the statistics count the step in CBF_STAT_ERRORS.
    The kernels after the scan do not read the unusable cell list (no scatter, identity order)."""
    import ctypes as C
    import os
    from cbf_amd import _lib
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcbf_scantimeout.so")
    L = C.CDLL(path)
    fn = L.cbf_lattice_step
    fn.restype, fn.argtypes = _lib.SIGNATURES["cbf_lattice_step"]
    W, H = 512, 512   # > one scan tile of cells, so some tile has a predecessor to wait for
    S = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=1), W, H)
    vel = torch.empty_like(S.pos)
    rc = fn(S.cp, C.byref(S.grid), W, H, 0, H, 0, H, _lib.ptr(S.pos), S.gain, S.T, _lib.ptr(S.pos), _lib.ptr(vel),
            _lib.ptr(S.u), _lib.ptr(S.status), _lib.ptr(S.nbr_count), 0, None, _lib.ptr(S.stats), _lib.ptr(S.ws),
            S.ws_bytes, _lib.stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    assert (S.status.cpu().numpy() == _lib.STATUS_WORKSPACE_ERROR).all()
    with pytest.raises(cbf_amd.CbfError):
        S.stats_summary()
    assert _lib.decode_stats(S.stats.cpu().numpy())["errors"] == 1


def test_allpairs_spilled_variant_is_bit_identical():
    """Round 1 recorded a `waves_per_eu = 8` all-pairs variant with wrong results and blamed the
    compiler.  The same request on the shipped all-pairs kernels (test build
    tests/_lib/libcbf_apwpe8.so, CBF_AP_WPE = 8: 64 VGPRs, 84-496 B of scratch per lane) must give
    the shipped kernels' and the oracle's results bit for bit, on the split (cfg3) and the unsplit
    path, with obstacles and the diagnostics."""
    import ctypes as C
    import os
    from cbf_amd import _lib
    V = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcbf_apwpe8.so"))
    split, full = V.cbf_filter_allpairs_split, V.cbf_filter_allpairs
    split.restype, split.argtypes = _lib.SIGNATURES["cbf_filter_allpairs_split"]
    full.restype, full.argtypes = _lib.SIGNATURES["cbf_filter_allpairs"]
    W, H, n_obs = 96, 64, 40
    pos = scenarios.lattice(W, H, seed=21)
    vel = coracle.consensus_lattice(W, H, 0, H, pos, 0.25)
    n = pos.shape[0]
    p = swarm.FilterParams()
    cp = p.c()
    tp, tv = _t(pos), _t(vel)
    ref = swarm.filter_swarm(p, tp, tv, n_obs, method="allpairs")
    want = coracle.filter_swarm(po.Params(15), pos, vel, n_obs)
    assert np.array_equal(ref["u"].cpu().numpy(), want["u"])
    ne = n - n_obs
    u = torch.empty((ne, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((ne,), dtype=torch.int32, device="cuda")
    cnt = torch.empty((ne,), dtype=torch.int32, device="cuda")
    wsb = _lib.lib.cbf_allpairs_workspace_size(n, ne)
    ws = torch.empty((wsb,), dtype=torch.uint8, device="cuda")
    assert split(cp, n, n_obs, _lib.ptr(tp), _lib.ptr(tv), n_obs, n, _lib.ptr(u), _lib.ptr(st), _lib.ptr(cnt),
                 _lib.ptr(ws), wsb, _lib.stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(u, ref["u"]) and torch.equal(st, ref["status"]) and torch.equal(cnt, ref["nbr_count"])
    u.zero_()
    assert full(cp, n, n_obs, _lib.ptr(tp), _lib.ptr(tv), n_obs, n, _lib.ptr(u), _lib.ptr(st), _lib.ptr(cnt),
                C.byref(_lib.CbfDiag()), _lib.stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(u, ref["u"]) and torch.equal(st, ref["status"]) and torch.equal(cnt, ref["nbr_count"])


@pytest.mark.parametrize("nominal", [None, ("random", 1.0, 5)])
def test_full_solve_placements_are_bit_identical(nominal):
    """The two placements of the full solve of the QPs solve_fast cannot settle (inline in the
    filter, queued for the one-lane queue kernel; cbf_params.solve_inline_max) and the automatic
    pick give the same results bit for bit over a chained rollout (positions, last-step controls and
    statuses, every statistics word), on the consensus lattice at spacing 0.2 and on cfg4r's random
    walk (10 % of the QPs through the full solve)."""
    W, H, steps = 160, 128, 8
    pos = scenarios.lattice(W, H, seed=13, spacing=0.2 if nominal is None else 0.22)
    runs = {}
    for placement in ("auto", "inline", "queued"):
        A = swarm.LatticeSwarm(pos, W, H, nominal=nominal, params=_fp(placement))
        A.run(steps)
        runs[placement] = _lattice_state(A)
        st = A.stats_summary()
        assert st["seidel"] > 0 and st["errors"] == 0
    for placement in ("inline", "queued"):
        for a, b in zip(runs["auto"], runs[placement]):
            assert np.array_equal(a, b), placement


def _oracle_window_step(pos, W, H, gain, threads=16):
    """One timestep of the whole W x H lattice by the C oracle, its egos split over `threads` ego
    ranges (the O(N) reference cull per ego, cross_and_rescue.py:141-150, on the host's cores)."""
    vel = coracle.consensus_lattice(W, H, 0, H, pos, gain)
    p = po.Params(15)
    bounds = np.linspace(0, W * H, threads + 1).astype(int)

    def run(k):
        return coracle.filter_swarm(p, pos, vel, 0, int(bounds[k]), int(bounds[k + 1]))
    with cf.ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(run, range(threads)))
    out = {key: np.concatenate([q[key] for q in parts]) for key in ("u", "status", "cnt")}
    return coracle.euler(pos, out["u"], 1 / 30), vel, out


@pytest.mark.parametrize("placement,cull", [("auto", "cells"), ("inline", "cells"), ("auto", "window")])
def test_large_window_run_vs_oracle_every_timestep(placement, cull):
    """The bench's timed path on a window above the inline threshold (1024 x 136 = 139,264 agents >
    131,072): the shipped cbf_lattice_run with stats = NULL -- auto places the full solves in the
    queue kernel, whose chained binning feeds the next timestep -- checked bit for bit against the
    oracle at EVERY timestep (nominal control, filtered control, status, neighbour count, and the
    positions they imply), through run(4, history=True) (every timestep's outputs stored) and a
    plain run(4) (the bench's form: outputs of the last timestep only).  "inline" forces the other
    placement on the same window; "window" runs the lattice-window cull (its queued path)."""
    W, H, steps = 1024, 136, 4
    pos = scenarios.lattice(W, H, seed=17)
    fp = _fp(placement)
    A = swarm.LatticeSwarm(pos, W, H, params=fp, cull=cull)
    A.collect_stats = False
    A.run(steps, history=True)
    B = swarm.LatticeSwarm(pos, W, H, params=fp, cull=cull)
    B.collect_stats = False
    B.run(steps)
    torch.cuda.synchronize()
    hv, hu, hs, hc = (t.cpu().numpy() for t in A.history(steps))
    ref = pos.copy()
    for t in range(steps):
        nxt, vel, out = _oracle_window_step(ref, W, H, scenarios.LATTICE_GAIN)
        assert np.array_equal(hv[t], vel), t
        assert np.array_equal(hu[t], out["u"]), t
        assert np.array_equal(hs[t], out["status"]), t
        assert np.array_equal(hc[t], out["cnt"]), t
        ref = nxt
    assert np.array_equal(A.pos.cpu().numpy(), ref)
    assert np.array_equal(B.pos.cpu().numpy(), ref)
    assert np.array_equal(B.u.cpu().numpy(), out["u"]) and np.array_equal(B.status.cpu().numpy(), out["status"])
    # the window holds full solves (the queue kernel has work under "auto")
    C = swarm.LatticeSwarm(pos, W, H, params=fp, cull=cull)
    C.run(steps)
    assert C.stats_summary()["seidel"] > 0


def _host_cells(pos, g):
    """Cell of every position, as cell_coord / cell_of compute it (floor((v - o) inv_h), clamped)."""
    def coord(v, o, n):
        f = np.floor((v - o) * g.inv_h)
        f = np.where(f >= 0.0, f, 0.0)
        return np.minimum(f, n - 1).astype(np.int64)
    return coord(pos[:, 1], g.y0, g.ny) * g.nx + coord(pos[:, 0], g.x0, g.nx)


@pytest.mark.parametrize("steps", [1, 6])
def test_cell_starts_full_size_equal_host_scan(steps):
    """The in-launch hand-off of k_lattice_scan_scatter (cells.hpp scan_tile: sc1 start stores and
    done words, sc1 loads by the scatter) at full size: after a build of the 1 M-agent lattice, every
    cell start equals the host's exclusive scan of the cell counts of the positions binned, the
    sorted indices are a permutation, and every sorted slot holds an agent of its own cell with its
    own position.  steps = 6: five timesteps first, so the bin pass walks the previous cell order."""
    import ctypes as C
    from cbf_amd import _lib
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=3)
    L = swarm.LatticeSwarm(pos, W, H)
    L.collect_stats = False
    if steps > 1:
        L.run(steps - 1)
    torch.cuda.synchronize()
    p_in = L.pos.cpu().numpy()
    L.build_phase()
    torch.cuda.synchronize()
    off = (C.c_int64 * 4)()
    ncell = _lib.lib.cbf_lattice_workspace_view(W, H, C.byref(L.grid), off)
    assert ncell == L.grid.nx * L.grid.ny
    ws = L.ws.cpu().numpy()
    start = ws[off[0]:off[0] + 4 * (ncell + 1)].view(np.int32)
    spos = ws[off[1]:off[1] + 16 * W * H].view(np.float64).reshape(-1, 2)
    sidx = ws[off[3]:off[3] + 4 * W * H].view(np.int32)
    cells = _host_cells(p_in, L.grid)
    counts = np.bincount(cells, minlength=ncell)
    want = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    assert np.array_equal(start.astype(np.int64), want)
    assert np.array_equal(np.sort(sidx), np.arange(W * H))
    assert np.array_equal(spos, p_in[sidx])
    slot_cell = np.repeat(np.arange(ncell), counts)
    assert np.array_equal(cells[sidx], slot_cell)


@pytest.mark.parametrize("spacing", [0.145, 0.2], ids=["cfg4", "cfg4f"])
def test_window_full_size_driver_timesteps_vs_oracle(spacing):
    """The driver's headline path at its own size and timesteps: the 1024 x 1024 lattice under the
    window cull through cbf_lattice_run with statistics off (bench.py cfg4 times timesteps 6-25 of
    this rollout), and cfg4f's (spacing 0.2: most QPs feasible, the branch of cbf.py:75-87 whose
    answer the reference defines; bench.py's feasible_regime record).  One run(25, history=True) stores every timestep's nominal control, filtered
    control, status and neighbour count; the input positions of every timestep follow from them by
    the Euler update (the device's own arithmetic, p + T u), and the plain run(25) -- the bench's
    form -- must end in the same positions.  At timesteps 6, 15 and 25, 512 sampled egos are
    checked against the oracle's O(N) reference cull and filter (cross_and_rescue.py:135-160):
    controls, statuses and neighbour counts bit for bit, nominal controls over the whole lattice."""
    W = H = 1024
    steps = 25
    pos = scenarios.lattice(W, H, seed=0, spacing=spacing)
    A = swarm.LatticeSwarm(pos, W, H, cull="window")
    A.collect_stats = False
    A.run(steps, history=True)
    torch.cuda.synchronize()
    hv, hu, hs, hc = (t.cpu().numpy() for t in A.history(steps))
    end_a = A.pos.cpu().numpy()
    del A
    B = swarm.LatticeSwarm(pos, W, H, cull="window")
    B.collect_stats = False
    B.run(steps)
    torch.cuda.synchronize()
    assert np.array_equal(B.pos.cpu().numpy(), end_a)
    del B
    p = pos.copy()
    rng = np.random.default_rng(25)
    optimal = 0
    for t in range(steps):
        if t + 1 in (6, 15, 25):
            vel = coracle.consensus_lattice(W, H, 0, H, p, scenarios.LATTICE_GAIN)
            assert np.array_equal(hv[t], vel), t + 1
            idx = rng.choice(W * H, 512, replace=False)
            for e, (ru, rst, rc) in zip(idx, _sample_oracle(p, vel, idx)):
                assert np.array_equal(hu[t][e], ru) and hs[t][e] == rst and hc[t][e] == rc, (t + 1, e)
                optimal += (rst & 0xFF) == 1
        p = coracle.euler(p, hu[t], 1 / 30)
    assert np.array_equal(p, end_a)
    if spacing == 0.2:  # the sample exercises the feasible (OPTIMAL) branch, not only the relaxation
        print(f"cfg4f sample: {optimal} of {3 * 512} sampled egos OPTIMAL")
        assert optimal >= 256, optimal
