"""Euclidean HOCBF barrier mode on the HIP path against the C / Python restatement (bit-exact)
and the reference-order cull (index sets bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

import cbf_amd  # noqa: E402
from cbf_amd import swarm  # noqa: E402
from oracle import coracle, pyoracle as po  # noqa: E402

from .test_hocbf_oracle import _cases  # noqa: E402

DEV = torch.device("cuda")


def _t(a, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=DEV)


def test_batch_vs_oracle():
    rng = np.random.default_rng(31)
    groups = {}
    for p, hp, r, obs, u0 in _cases(rng, 600):
        groups.setdefault((p.max_speed, p.dmin, hp.alpha1, hp.alpha2), []).append((p, hp, r, obs, u0))
    n_checked = 0
    for (ms, dmin, a1, a2), cases in groups.items():
        c = cbf_amd.ControlBarrierFunction(ms, dmin=dmin, barrier="euclidean_hocbf", alpha1=a1, alpha2=a2)
        R = np.array([cs[2] for cs in cases])
        U0 = np.array([cs[4] for cs in cases])
        u, st, x = c.get_safe_control_batch(_t(R), [_t(cs[3].reshape(-1, 4)) for cs in cases], _t(U0), return_x=True)
        u, st, x = u.cpu().numpy(), st.cpu().numpy(), x.cpu().numpy()
        for t, (p, hp, r, obs, u0) in enumerate(cases):
            ref = coracle.filter_one_hocbf(p, hp, r, obs, u0)
            assert st[t] & 0xFF == ref["status"] and st[t] >> 8 == ref["iters"], t
            assert np.array_equal(u[t], ref["u"]) and np.array_equal(x[t], ref["x"]), t
            n_checked += 1
    assert n_checked == 600


def test_single_call_surface():
    c = cbf_amd.ControlBarrierFunction(15, barrier="euclidean_hocbf")
    r = np.array([0.0, 0.0, 0.04, 0.0])
    u = c.get_safe_control(r, np.array([[0.25, 0.0, 0.0, 0.0]]), np.zeros((4, 4)), np.zeros((4, 2)), [0.0, 0.0])
    ref = po.filter_one_hocbf(po.Params(15), po.HocbfParams(1.0, 1.0), r, [[0.25, 0.0, 0.0, 0.0]], [0.0, 0.0])
    assert isinstance(u, np.ndarray) and u.shape == (2,)
    assert np.array_equal(u, np.array(ref["u"])) and u[0] < 0
    with pytest.raises(ValueError):
        cbf_amd.ControlBarrierFunction(15, barrier="nope")


@pytest.mark.parametrize("n,n_obs,spread", [(50, 10, 0.4), (2000, 200, 3.0)])
def test_swarm_vs_oracle(n, n_obs, spread):
    rng = np.random.default_rng(n)
    p, hp = po.Params(15), po.HocbfParams(1.0, 2.0)
    pos = rng.uniform(-spread, spread, (n, 2))
    vel = rng.normal(0, 0.3, (n, 2))
    pos[n_obs + 3] = pos[n_obs + 5]               # coincident agents: excluded from each other
    pos[n_obs + 7] = pos[n_obs + 6] + [0.2, 0.0]  # exactly at the cull radius
    out = swarm.filter_swarm_hocbf(swarm.FilterParams(), _t(pos), _t(vel), n_obs, alpha=(1.0, 2.0), kmax=4,
                                   return_x=True)
    ref = coracle.filter_swarm_hocbf(p, hp, pos, vel, n_obs)
    assert np.array_equal(out["nbr_count"].cpu().numpy(), ref["cnt"])
    assert np.array_equal(out["u"].cpu().numpy(), ref["u"])
    assert np.array_equal(out["status"].cpu().numpy(), ref["status"])
    assert np.array_equal(out["x"].cpu().numpy(), ref["x"])
    # neighbour index sets in reference order (cross_and_rescue.py:141-150)
    idx = out["nbr_idx"].cpu().numpy()
    for k in range(0, n - n_obs, max(1, (n - n_obs) // 50)):
        want = po.cull_one(p, pos, n_obs, n_obs + k)
        assert idx[k, :len(want)].tolist() == want and (idx[k, len(want):] == -1).all()


def test_overflow_status_when_kmax_too_small():
    rng = np.random.default_rng(3)
    pos = rng.uniform(-0.1, 0.1, (40, 2))
    vel = np.zeros((40, 2))
    P = _t(pos)
    cnt = torch.empty(40, dtype=torch.int32, device=DEV)
    idx = torch.empty((40, 2), dtype=torch.int32, device=DEV)
    from cbf_amd._lib import C, CbfHocbf, lib, ptr, stream_handle
    cp = swarm.FilterParams().c()
    assert lib.cbf_cull_allpairs(cp, 40, 0, ptr(P), 0, 40, 2, ptr(idx), ptr(cnt), stream_handle()) == 0
    u = torch.empty((40, 2), dtype=torch.float64, device=DEV)
    st = torch.empty(40, dtype=torch.int32, device=DEV)
    ws = torch.empty(lib.cbf_hocbf_workspace_size(80), dtype=torch.uint8, device=DEV)
    hp = CbfHocbf(1.0, 1.0)
    assert lib.cbf_filter_indexed_hocbf(cp, C.byref(hp), 40, ptr(P), ptr(_t(vel)), 0, 40, 2, ptr(idx), ptr(cnt),
                                        ptr(u), ptr(st), None, ptr(ws), ws.numel(), stream_handle()) == 0
    assert (st.cpu().numpy() == cbf_amd.STATUS_NBR_OVERFLOW).all()


@pytest.mark.parametrize("alpha", [(1.0, 1.0), (2.0, 0.5)])
def test_lattice_step_hocbf_vs_oracle(alpha):
    """The cfg4-shape fused step in HOCBF mode (nominal + cell list + HOCBF filter + clip + Euler),
    3 steps (the last two replayed from a hipGraph), bit-exact vs the oracle's all-pairs loop."""
    from cbf_amd import scenarios
    W = H = 48
    pos = scenarios.lattice(W, H, seed=7)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf", alpha=alpha)
    p, hp = po.Params(15), po.HocbfParams(*alpha)
    ref_pos = pos.copy()
    for step in range(3):
        if step == 1:
            L.capture()
            L.pos.copy_(torch.as_tensor(ref_pos, device=DEV))  # capture ran one step: rewind
        L.step()
        torch.cuda.synchronize()
        vel = coracle.consensus_lattice(W, H, 0, H, ref_pos, scenarios.LATTICE_GAIN)
        ref = coracle.filter_swarm_hocbf(p, hp, ref_pos, vel, 0)
        ref_pos = coracle.euler(ref_pos, ref["u"], 1 / 30)
        st = L.status.cpu().numpy()
        assert not ((st & 0xFF) == cbf_amd.STATUS_NBR_OVERFLOW).any()
        assert np.array_equal(L.nbr_count.cpu().numpy(), ref["cnt"]), step
        assert np.array_equal(st, ref["status"]), step
        assert np.array_equal(L.u.cpu().numpy(), ref["u"]), step
        assert np.array_equal(L.pos.cpu().numpy(), ref_pos), step


@pytest.mark.parametrize("spacing", [0.09, 0.075])
def test_lattice_hocbf_dense_queue(spacing):
    """Dense lattices: egos with 9..24 neighbours take the queue + wide kernel
    (k_lattice_filter_hocbf_wide), more than 24 report NBR_OVERFLOW with u = u0.  Teacher-forced
    3 steps (the last two replayed from a hipGraph, so the queue is emptied and refilled),
    bit-exact vs the oracle on every ego the cap admits."""
    from cbf_amd import scenarios
    W = H = 40
    pos = scenarios.lattice(W, H, seed=3, spacing=spacing)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
    p, hp = po.Params(15), po.HocbfParams(1.0, 1.0)
    seen_wide = seen_over = 0
    for step in range(3):
        if step == 1:
            L.capture()
        cur = L.pos.cpu().numpy().copy()
        L.step()
        torch.cuda.synchronize()
        vel = coracle.consensus_lattice(W, H, 0, H, cur, scenarios.LATTICE_GAIN)
        ref = coracle.filter_swarm_hocbf(p, hp, cur, vel, 0)
        cnt = L.nbr_count.cpu().numpy()
        st = L.status.cpu().numpy()
        u = L.u.cpu().numpy()
        assert np.array_equal(cnt, ref["cnt"]), step
        over = cnt > 24
        seen_wide += int(((cnt > 8) & ~over).sum())
        seen_over += int(over.sum())
        assert np.array_equal(st[~over], ref["status"][~over]), step
        assert ((st[over] & 0xFF) == cbf_amd.STATUS_NBR_OVERFLOW).all()
        want_u = np.where(over[:, None], vel, ref["u"])
        assert np.array_equal(u, want_u), step
        assert np.array_equal(L.pos.cpu().numpy(), coracle.euler(cur, want_u, 1 / 30)), step
    assert seen_wide > 0
    if spacing < 0.08:
        assert seen_over > 0


@pytest.mark.parametrize("barrier", ["reference", "euclidean_hocbf"])
def test_lattice_advance_twice_without_build(barrier):
    """The queue kernels empty their queue when done: an advance run again on the same build
    gives the same outputs and counts exactly the same solves (no stale queue entries)."""
    from cbf_amd import scenarios
    W = H = 40
    pos = scenarios.lattice(W, H, seed=5, spacing=0.085)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier=barrier)
    p0 = L.pos.clone()
    L.build_phase()
    outs, counts = [], []
    for _ in range(3):
        L.pos.copy_(p0)
        L.reset_solves()
        L.advance_phase()
        torch.cuda.synchronize()
        outs.append((L.pos.cpu().numpy(), L.u.cpu().numpy(), L.status.cpu().numpy()))
        counts.append(L.solves_total())
    assert counts[0] > 0 and counts[0] == counts[1] == counts[2]
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


def test_lattice_hocbf_run_graph_equals_steps():
    """HOCBF mode's run(steps): `steps` timesteps captured as one hipGraph (capture(steps)) give
    the same positions, controls, statuses and solve count as as many step() calls, and as the
    eager run(steps); the per-step-outputs form is the reference barrier's only."""
    from cbf_amd import scenarios
    W = H = 40
    pos = scenarios.lattice(W, H, seed=11, spacing=0.1)  # some egos take the wide kernel
    A = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
    B = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
    C = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
    for _ in range(7):
        A.step()
    snap = B.snapshot()
    B.capture(steps=5)   # its warm-up launch advances B: rewind
    B.restore(snap)
    B.reset_solves()
    B.run(5)
    B.run(2)             # (no graph of 2 steps: eager)
    C.run(7)
    torch.cuda.synchronize()
    for S in (B, C):
        assert np.array_equal(A.pos.cpu().numpy(), S.pos.cpu().numpy())
        assert np.array_equal(A.u.cpu().numpy(), S.u.cpu().numpy())
        assert np.array_equal(A.status.cpu().numpy(), S.status.cpu().numpy())
        assert A.solves_total() == S.solves_total()
    assert int((A.nbr_count > 8).sum()) > 0
    with pytest.raises(ValueError):
        B.run(3, history=True)


@pytest.mark.parametrize("spacing,poison", [(0.145, False), (0.1, False), (0.145, True)])
def test_lattice_hocbf_certificate_skip_is_bit_identical(spacing, poison):
    """The HOCBF kernels skip a first relaxation pass that a three-row Farkas certificate proves
    infeasible (hocbf_cert / hocbf_cert_wave).  Against the test build that runs every pass
    (tests/_lib/libcbf_hocbfnocert.so, CBF_HOCBF_CERT=0), advance by advance on the same cell list:
    positions, controls, statuses (relaxation counts included) and neighbour counts bit for bit,
    on the cfg4 spacing (most egos certified) and a denser one (wide-kernel egos too)."""
    import ctypes as C
    import os
    from cbf_amd import _lib, scenarios
    V = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcbf_hocbfnocert.so"))
    adv = V.cbf_lattice_advance_hocbf
    adv.restype, adv.argtypes = _lib.SIGNATURES["cbf_lattice_advance_hocbf"]
    W = H = 96
    pos = scenarios.lattice(W, H, seed=4, spacing=spacing)
    if poison:  # non-finite agents: their neighbours' rows are NaN / inf (never settled by the certificate)
        pos[W * 40 + 40] = (np.nan, 0.5)
        pos[W * 60 + 20] = (np.inf, -np.inf)
    L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
    relaxed = wide = 0
    for _ in range(6):
        L.build_phase()
        p0 = L.pos.clone()
        L.advance_phase()
        torch.cuda.synchronize()
        got = [t.clone() for t in (L.pos, L.u, L.status, L.nbr_count)]
        L.pos.copy_(p0)
        assert adv(L.cp, C.byref(L.hp), C.byref(L.grid), W, H, 0, H, 0, H, _lib.ptr(L.pos), L.T, _lib.ptr(L.pos),
                   _lib.ptr(L.u), _lib.ptr(L.status), _lib.ptr(L.nbr_count), 0, None, None, _lib.ptr(L.ws),
                   L.ws_bytes, _lib.stream_handle()) == 0
        torch.cuda.synchronize()
        for a, b in zip(got, (L.pos, L.u, L.status, L.nbr_count)):
            assert torch.equal(a.cpu().view(torch.int64) if a.dtype == torch.float64 else a.cpu(),
                               b.cpu().view(torch.int64) if b.dtype == torch.float64 else b.cpu())  # (NaN bits too)
        st = L.status.cpu().numpy()
        relaxed += int(((st & 0xFF) == cbf_amd.STATUS_RELAXED).sum())
        wide += int((L.nbr_count > 8).sum())
    assert relaxed > 0
    if spacing < 0.12:
        assert wide > 0
