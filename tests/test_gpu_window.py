"""The lattice-window cull (include/cbf_amd.h CBF_RUN_WINDOW_CULL, cbf_amd/csrc/window.hip) against
the C oracle's O(N) reference cull (cross_and_rescue.py:141-150) on swarms chosen to break every
shortcut the window takes: agents far from their lattice site, rows out of x order, a dense clump
that overflows the hit list, coincident agents, non-finite positions, narrow and short lattices.
The cull decides only which candidates are tested; results must be the cell list's and the
oracle's bit for bit whatever the swarm looks like."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU boxes but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from cbf_amd import scenarios, swarm  # noqa: E402
from oracle import coracle, pyoracle as po  # noqa: E402
from tests import paramsets  # noqa: E402

GAIN = 0.25
WINDOW_ONLY = ("win_walks", "guard_stalls")   # statistics words only the window cull counts


def _stats_row(st):
    return np.array([st[k] for k in sorted(st) if k not in WINDOW_ONLY], dtype=object)


def _oracle_rollout(pos, W, H, steps, pset="callers"):
    ref = pos.copy()
    outs = []
    p = paramsets.oracle_params(pset)
    for _ in range(steps):
        vel = coracle.consensus_lattice(W, H, 0, H, ref, GAIN)
        out = coracle.filter_swarm(p, ref, vel, 0)
        ref = coracle.euler(ref, out["u"], 1 / 30)
        outs.append((vel, out, ref.copy()))
    return outs


def _check_steps(pos, W, H, steps, placement="auto", equal_nan=False, pset="callers", stats=True):
    """step() of the window cull and of the cell list, every timestep against the oracle.  stats=False:
    the statistics-free kernels (with queued QPs, the window filter's timed instantiation, the one
    the bench runs)."""
    runs = [swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=paramsets.filter_params(pset, solve_placement=placement),
                               cull=c)
            for c in ("window", "cells")]
    for L in runs:
        L.collect_stats = stats
    for t, (vel, out, ref) in enumerate(_oracle_rollout(pos, W, H, steps, pset)):
        for L in runs:
            L.step()
            torch.cuda.synchronize()
            tag = (L.cull, t)
            assert np.array_equal(L.vel.cpu().numpy(), vel, equal_nan=equal_nan), tag
            assert np.array_equal(L.u.cpu().numpy(), out["u"], equal_nan=equal_nan), tag
            assert np.array_equal(L.status.cpu().numpy(), out["status"]), tag
            assert np.array_equal(L.nbr_count.cpu().numpy(), out["cnt"]), tag
            assert np.array_equal(L.pos.cpu().numpy(), ref, equal_nan=equal_nan), tag
    return runs


@pytest.mark.parametrize("pset", paramsets.NAMES)
@pytest.mark.parametrize("placement,stats", [("inline", True), ("queued", True), ("queued", False)])
def test_window_scrambled_lattice_vs_oracle(placement, stats, pset):
    """Agents swapped with far-away ones (a lattice index no longer says where an agent is), so
    the row and column guards fail for their neighbours and those egos walk their rows outward;
    plus coincident agents (s = 0: not neighbours) and an exact-cutoff pair.  pset: the callers'
    parameters or others (tests/paramsets.py; the 0.3 cull radius reaches beyond the staged tile)."""
    W, H = 64, 48
    pos = scenarios.lattice(W, H, seed=21)
    rng = np.random.default_rng(4)
    a = rng.choice(W * H, 40, replace=False)
    b = rng.choice(W * H, 40, replace=False)
    pos[a], pos[b] = pos[b].copy(), pos[a].copy()
    pos[100] = pos[101]                        # coincident pair
    pos[300] = pos[301] + np.array([0.2, 0.0])  # s == 0.04 exactly is out (sqrt(s) < 0.2 fails)
    runs = _check_steps(pos, W, H, 5, placement, pset=pset, stats=stats)
    walks, _ = runs[0].window_counters()
    assert walks > 0


def test_window_dense_clump_overflows_hit_list():
    """25 agents packed in a 0.1-wide square: > 16 hits per ego (the hit list's cap), so those
    egos take the direct-assembly walk; the rows they sit in are far out of x order."""
    W, H = 48, 40
    pos = scenarios.lattice(W, H, seed=22)
    rng = np.random.default_rng(5)
    idx = rng.choice(W * H, 25, replace=False)
    pos[idx] = np.array([1.0, 1.0]) + 0.1 * rng.random((25, 2))
    runs = _check_steps(pos, W, H, 4)
    assert runs[0].nbr_count.cpu().numpy().max() > 16


def test_window_unsorted_rows_vs_oracle():
    """Every other lattice row reversed in x (its column extents then exclude nothing nearby):
    correct, by the unbounded walk, however un-lattice-like."""
    W, H = 40, 24
    pos = scenarios.lattice(W, H, seed=23).reshape(H, W, 2)
    pos[1::2] = pos[1::2, ::-1]
    _check_steps(pos.reshape(-1, 2).copy(), W, H, 3)


@pytest.mark.parametrize("W,H", [(4, 1), (4, 6), (5, 3), (70, 9), (130, 2), (2048, 2)])
def test_window_edge_shapes(W, H):
    """Narrow, short and wide lattices: candidates and sentinels beyond the row ends and beyond the
    first / last row, a window of one row, rows of several waves."""
    pos = scenarios.lattice(W, H, seed=24, spacing=0.15)
    _check_steps(pos, W, H, 3)


@pytest.mark.parametrize("placement,stats", [("auto", True), ("inline", False), ("queued", True), ("queued", False)])
def test_window_nonfinite_positions_match_cells(placement, stats):
    """Non-finite positions (NaN, +-inf) never pass the cull test and are left out of the guards'
    extents; the window cull then gives the cell list's results bit for bit (NaNs compared as
    equal), with the QPs solved inline and queued.  The tile forms a quadrant's presence from its
    minimum (a NaN or +inf row leaves it absent) where the cell list's assembly marks every hit
    present; the solve is the same either way (a +inf plane never binds), so the egos next to a
    non-finite neighbour -- a NaN nominal control makes their rows NaN -- must agree exactly."""
    W, H = 48, 32
    pos = scenarios.lattice(W, H, seed=25)
    pos[10] = [np.nan, 0.3]
    pos[500] = [np.inf, pos[500, 1]]
    pos[900] = [pos[900, 0], -np.inf]
    fp = paramsets.filter_params("callers", solve_placement=placement)
    A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=fp, cull="window")
    B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=fp, cull="cells")
    A.collect_stats = B.collect_stats = stats
    near = [9, 11, 10 + W, 499, 501, 500 - W, 899, 901, 900 + W]
    for _ in range(3):
        A.step()
        B.step()
        torch.cuda.synchronize()
        for x, y in ((A.pos, B.pos), (A.u, B.u), (A.vel, B.vel)):
            assert np.array_equal(x.cpu().numpy(), y.cpu().numpy(), equal_nan=True)
        assert torch.equal(A.status, B.status) and torch.equal(A.nbr_count, B.nbr_count)
        assert np.array_equal(A.u[near].cpu().numpy(), B.u[near].cpu().numpy(), equal_nan=True)
        assert torch.equal(A.status[near], B.status[near])


@pytest.mark.parametrize("nominal", [None, ("random", 1.0, 5)])
def test_window_run_equals_cells_run(nominal):
    """run() (odd and even step counts: the ping-pong through the workspace), a hipGraph of run(4)
    and the statistics are the cell list's bit for bit, on the consensus lattice and on cfg4r's
    random walk (which scrambles the lattice: more and more egos walk their rows outward)."""
    W, H = 160, 128
    pos = scenarios.lattice(W, H, seed=26, spacing=0.145 if nominal is None else 0.22)
    res = {}
    for cull in ("cells", "window"):
        A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, nominal=nominal, cull=cull)
        A.run(3)
        A.capture(steps=4)   # warm-up launch: timesteps 4-7
        A.run(4)             # replay: 8-11
        A.run(1)
        torch.cuda.synchronize()
        st = A.stats_summary()
        res[cull] = [t.cpu().numpy() for t in (A.pos, A.vel, A.u, A.status, A.nbr_count)] + [_stats_row(st)]
        if cull == "window":
            walks = st["win_walks"]
    for a, b in zip(res["cells"], res["window"]):
        assert np.array_equal(a, b)
    # the random walk scrambles the lattice: egos walk their rows (CBF_STAT_WIN_WALKS counts them)
    if nominal is not None:
        assert walks > 0


def test_window_advance_phase_marked_equals_step():
    """build_phase() + advance_phase(mark) of the window cull (the bench's measurement hook) ==
    one step(), and the event lands inside the advance."""
    W, H = 96, 64
    pos = scenarios.lattice(W, H, seed=27, spacing=0.2)
    A = swarm.LatticeSwarm(pos, W, H, cull="window")
    B = swarm.LatticeSwarm(pos, W, H, cull="window")
    A.step()
    B.build_phase()
    a, m, b = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    m.record()
    a.record()
    B.advance_phase(mark=m)
    b.record()
    torch.cuda.synchronize()
    assert torch.equal(A.pos, B.pos) and torch.equal(A.u, B.u) and torch.equal(A.status, B.status)
    assert torch.equal(A.vel, B.vel)
    assert 0 <= a.elapsed_time(m) <= a.elapsed_time(b)


def test_window_full_size_cfg4_equals_cells():
    """cfg4 at full size (1024 x 1024), 12 timesteps: the window cull's rollout == the cell list's
    (which the oracle tests pin) bit for bit, statistics included."""
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0)
    res = {}
    for cull in ("cells", "window"):
        A = swarm.LatticeSwarm(pos, W, H, cull=cull)
        A.run(12)
        torch.cuda.synchronize()
        st = A.stats_summary()
        res[cull] = [t.cpu().numpy() for t in (A.pos, A.vel, A.u, A.status, A.nbr_count)] + [_stats_row(st)]
        del A
    for a, b in zip(res["cells"], res["window"]):
        assert np.array_equal(a, b)


def test_window_guard_words_never_ready():
    """A row-guard word that never carries the build's token (the first block's hand-off not seen;
    forced for every word by the test build tests/_lib/libcbf_winnowait.so, CBF_WIN_SPIN_LIMIT =
    -1) reads as the worst bound (every row a candidate row): every ego then walks all rows, and
    the results are the shipped library's bit for bit, on the scrambled lattice."""
    import ctypes as C
    import os
    from cbf_amd import _lib
    V = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcbf_winnowait.so"))
    fn = V.cbf_lattice_run_ex
    fn.restype, fn.argtypes = _lib.SIGNATURES["cbf_lattice_run_ex"]
    W, H = 64, 48
    pos = scenarios.lattice(W, H, seed=21)
    rng = np.random.default_rng(4)
    a = rng.choice(W * H, 40, replace=False)
    b = rng.choice(W * H, 40, replace=False)
    pos[a], pos[b] = pos[b].copy(), pos[a].copy()
    A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="window")
    B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="window")
    A.run(3)
    rc = fn(B.cp, C.byref(B.grid), W, H, _lib.ptr(B.pos), B.gain, B.T, 3, _lib.ptr(B.vel), _lib.ptr(B.u),
            _lib.ptr(B.status), _lib.ptr(B.nbr_count), B._st(), _lib.ptr(B.ws), B.ws_bytes, _lib.RUN_WINDOW_CULL,
            _lib.stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    for x, y in ((A.pos, B.pos), (A.u, B.u), (A.vel, B.vel), (A.status, B.status), (A.nbr_count, B.nbr_count)):
        assert torch.equal(x, y)
    sa, sb = A.stats_summary(), B.stats_summary()
    assert _stats_row(sa).tolist() == _stats_row(sb).tolist()
    # the degradation is visible: every word read as the worst bound, and every ego walked
    assert sa["guard_stalls"] == 0 and sb["guard_stalls"] > 0
    assert sb["win_walks"] == 3 * W * H > sa["win_walks"]
    ca, cb = A.window_counters(), B.window_counters()
    assert cb == (sb["win_walks"], sb["guard_stalls"]) and ca == (sa["win_walks"], 0)


@pytest.mark.parametrize("cull", ["window", "cells"])
def test_queued_events_equal_in_place(cull):
    """The queued form settles a QP's one-event stage in the filter wave only where more than
    kEventInPlace lanes need it, and queues the others whole (lattice_ego.hpp ego_finish).  The
    test build tests/_lib/libcbf_evqueue.so (CBF_EVENT_IN_PLACE = 64) queues every such QP: on the
    random-walk regime, where most QPs take a Seidel event, the results and the rollout statistics
    (CBF_STAT_SEIDEL: the QPs solve_fast cannot settle, counted by the queue kernel) are the
    shipped library's bit for bit.  A 48-column tile queues up to 384 QPs into a sub-queue sized
    for 256 (CellWs::subq_cap), so the full-sub-queue hand-off (subq_append) is exercised too."""
    import ctypes as C
    import os
    from cbf_amd import _lib
    V = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcbf_evqueue.so"))
    fn = V.cbf_lattice_run_ex
    fn.restype, fn.argtypes = _lib.SIGNATURES["cbf_lattice_run_ex"]
    W, H, steps = 48, 40, 4
    pos = scenarios.lattice(W, H, seed=5, spacing=0.22)
    kw = dict(nominal=("random", 1.0, 3), cull=cull, params=swarm.FilterParams(solve_placement="queued"))
    A = swarm.LatticeSwarm(pos, W, H, **kw)
    B = swarm.LatticeSwarm(pos, W, H, **kw)
    A.run(steps)
    flags = _lib.RUN_WINDOW_CULL if cull == "window" else 0
    rc = fn(B.cp, C.byref(B.grid), W, H, _lib.ptr(B.pos), B.gain, B.T, steps, _lib.ptr(B.vel), _lib.ptr(B.u),
            _lib.ptr(B.status), _lib.ptr(B.nbr_count), B._st(), _lib.ptr(B.ws), B.ws_bytes, flags,
            _lib.stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    for x, y in ((A.pos, B.pos), (A.u, B.u), (A.vel, B.vel), (A.status, B.status), (A.nbr_count, B.nbr_count)):
        assert torch.equal(x, y)
    sa, sb = A.stats_summary(), B.stats_summary()
    assert sa == sb
    assert sa["seidel"] > 0 and sa["binding"] > 0.5 * sa["solves"]


@pytest.mark.parametrize("cull", ["window", "cells"])
def test_timed_advance_equals_marked(cull):
    """advance_phase(timing=...) (cbf_lattice_*advance_timed: the filter launched with
    hipExtLaunchKernel start / stop events, bench.py's kernel timing) gives the plain advance's
    results bit for bit, and its events time the filter inside the advance call's span."""
    W, H = 256, 192
    pos = scenarios.lattice(W, H, seed=28)
    A = swarm.LatticeSwarm(pos, W, H, cull=cull)
    B = swarm.LatticeSwarm(pos, W, H, cull=cull)
    for L in (A, B):
        L.build_phase()
    a, b, fs, fe, m = (torch.cuda.Event(enable_timing=True) for _ in range(5))
    fs.record()
    fe.record()
    m.record()
    A.advance_phase(mark=m)
    a.record()
    B.advance_phase(timing=(fs, fe))
    b.record()
    torch.cuda.synchronize()
    for x, y in ((A.pos, B.pos), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count)):
        assert torch.equal(x, y)
    t = fs.elapsed_time(fe)
    assert 0 < t <= a.elapsed_time(b)


def test_window_separate_guard_equals_in_filter():
    """cbf_params.launch_flags CBF_LAUNCH_SEPARATE_GUARD (FilterParams(window_guard="separate"):
    the row guard from the one-block scan kernel after the build, for ranks time-sharing a GPU)
    gives the in-filter hand-off's results bit for bit, run() and step(), scrambled lattice."""
    W, H = 64, 48
    pos = scenarios.lattice(W, H, seed=29)
    rng = np.random.default_rng(6)
    a, b = rng.choice(W * H, 30, replace=False), rng.choice(W * H, 30, replace=False)
    pos[a], pos[b] = pos[b].copy(), pos[a].copy()
    res = []
    for g in ("in_filter", "separate"):
        L = swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=swarm.FilterParams(window_guard=g), cull="window")
        L.run(3)
        L.step()
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (L.pos, L.vel, L.u, L.status, L.nbr_count)])
    for x, y in zip(*res):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("build_guard,advance_guard", [("in_filter", "separate"), ("separate", "in_filter")])
def test_window_guard_mode_follows_the_build(build_guard, advance_guard):
    """A build and an advance whose cbf_params disagree on CBF_LAUNCH_SEPARATE_GUARD: the filter
    follows the build's choice recorded in the workspace header (window.hip kWinModeWord), so it
    never reads the other form's words (token-tagged fp32 words left by an earlier in-filter
    timestep read as doubles would drop neighbours).  Every timestep equals the cell list's."""
    W, H = 64, 48
    pos = scenarios.lattice(W, H, seed=31)
    rng = np.random.default_rng(8)
    a, b = rng.choice(W * H, 30, replace=False), rng.choice(W * H, 30, replace=False)
    pos[a], pos[b] = pos[b].copy(), pos[a].copy()
    A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=swarm.FilterParams(window_guard=advance_guard), cull="window")
    B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="cells")
    cp_build = swarm.FilterParams(window_guard=build_guard).c()
    cp_adv = A.cp
    for t in range(4):
        if t % 2 == 0:
            A.step()                  # both phases in the advance's mode: its words stay in the area
        else:
            A.cp = cp_build
            A.build_phase()
            A.cp = cp_adv
            A.advance_phase()
        B.step()
        torch.cuda.synchronize()
        for x, y in ((A.pos, B.pos), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count)):
            assert torch.equal(x, y), t


@pytest.mark.parametrize("guard", ["in_filter", "separate"])
@pytest.mark.parametrize("W,H", [(16, 1100), (2048, 6)])
def test_window_many_rows_and_widest_rows(W, H, guard):
    """More than 1,024 candidate rows (the row-guard scans run several chunks: 1,024 rows per
    chunk in both the in-filter and the separate form) and the widest rows the window cull takes
    (k_window_prep's 8-column-per-thread instantiation): every timestep equals the cell list's
    and, for the tall lattice, the oracle's."""
    pos = scenarios.lattice(W, H, seed=32, spacing=0.15)
    fp = swarm.FilterParams(window_guard=guard)
    A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, params=fp, cull="window")
    B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="cells")
    ref = pos.copy()
    for t in range(3):
        A.step()
        B.step()
        torch.cuda.synchronize()
        for x, y in ((A.pos, B.pos), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count)):
            assert torch.equal(x, y), t
        if W == 16:
            vel = coracle.consensus_lattice(W, H, 0, H, ref, GAIN)
            out = coracle.filter_swarm(po.Params(15), ref, vel, 0)
            ref = coracle.euler(ref, out["u"], 1 / 30)
            assert np.array_equal(A.u.cpu().numpy(), out["u"]) and np.array_equal(A.pos.cpu().numpy(), ref), t
    A.run(3)
    B.run(3)
    torch.cuda.synchronize()
    assert torch.equal(A.pos, B.pos)


def test_window_auto_switches_to_cells_when_the_swarm_scrambles():
    """LatticeSwarm(cull="auto"): the window cull while the swarm stays lattice-like, the cell list
    once the walks (CBF_STAT_WIN_WALKS, cbf_lattice_window_counters) pass AUTO_WALK_FRACTION of
    the egos per timestep.  On cfg4r's random walk (which scrambles x along every row within a few
    timesteps) it switches; on the consensus lattice it does not; either way the rollout equals the
    cell list's bit for bit."""
    W, H = 160, 128
    for nominal, spacing, switch in ((("random", 1.0, 5), 0.22, True), (None, 0.145, False)):
        pos = scenarios.lattice(W, H, seed=33, spacing=spacing)
        A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, nominal=nominal, cull="auto")
        B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, nominal=nominal, cull="cells")
        assert A.cull == "window"
        for _ in range(12):
            A.run(4)
            torch.cuda.synchronize()   # lets the non-blocking look see each copy
        B.run(48)
        torch.cuda.synchronize()
        assert (A.cull == "cells") == switch, (nominal, A._auto)
        for x, y in ((A.pos, B.pos), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count)):
            assert torch.equal(x, y), nominal
        walks, stalls = A.window_counters()
        print(f"auto cull, nominal {nominal}: last walk fraction {A._auto.get('last_fraction')}, "
              f"walks {walks}, stalls {stalls}, switched after {A._auto.get('switched_after')}")
        assert stalls == 0 and (walks > 0 if switch else True)


def test_window_auto_baseline_after_checkpoint_and_capture(tmp_path):
    """cull="auto" after a restore and a capture: the workspace header's walk counter (kWinWalkWord,
    word 20) carries walks _auto_check never counted -- the saved rollout's whole history, the
    capture's warm-up launch -- so the first look after either only sets the baseline.  A consensus
    lattice whose restored header claims 10^9 earlier walks must stay on the window cull, and its
    rollout equals the cell list's bit for bit."""
    W, H = 160, 128
    pos = scenarios.lattice(W, H, seed=34, spacing=0.145)
    A = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="auto")
    B = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="cells")
    A.run(4)
    torch.cuda.synchronize()
    A.ws[80:88] = torch.tensor([10 ** 9], dtype=torch.int64).view(torch.uint8).to(A.ws.device)
    path = str(tmp_path / "auto.npz")
    A.save_checkpoint(path)
    R = swarm.LatticeSwarm.from_checkpoint(path)
    assert R.cull_mode == "auto" and R.cull == "window" and R._auto["base"] is None
    for _ in range(6):
        R.run(4)
        torch.cuda.synchronize()
    R.collect_stats = False
    R.capture(steps=4)  # the warm-up launch adds 4 timesteps outside _auto_check
    for _ in range(6):
        R.run(4)
        torch.cuda.synchronize()
    assert R.cull == "window", R._auto
    B.run(4 + 24 + 4 + 24)
    torch.cuda.synchronize()
    for x, y in ((R.pos, B.pos), (R.u, B.u), (R.status, B.status)):
        assert torch.equal(x, y)
    assert R._auto.get("last_fraction") is not None and R._auto["last_fraction"] < R.AUTO_WALK_FRACTION
