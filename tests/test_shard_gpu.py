"""Sharded lattice step on the HIP path: 2 and 3 ranks rehearsed on one GPU (gloo, host-staged
exchange), with 1 and 4 sub-steps per exchange (6 steps: the last cycle is partial), compared
bit-for-bit with the CPU oracle's rollout of the whole lattice (and with the single-GPU step)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, W, R, steps, q, k=4, graph=False, run=False, nominal=None, exchange="neighbour",
            placement="auto", cull="cells"):
    try:
        _work(rank, ws, port, W, R, steps, q, k, graph, run, nominal, exchange, placement, cull)
    except BaseException as e:   # report instead of leaving the test waiting on the queue
        q.put((rank, "error", repr(e)))
        raise


def _spacing(nominal):
    from cbf_amd import scenarios
    return scenarios.LATTICE_SPACING if nominal is None else 0.22   # random walk: the cfg4r spacing


def _work(rank, ws, port, W, R, steps, q, k, graph, run, nominal, exchange, placement, cull):
    import datetime
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=60))
    from cbf_amd.shard import ShardedLattice
    from cbf_amd.swarm import FilterParams
    # the random walk's RELAXED QPs can move an agent up to T * max_speed = 0.5 per step (the
    # guard catches it with the default 4-row halo): 10 rows per sub-step cover it
    S = ShardedLattice(W, R, seed=7, substeps=k, nominal=nominal, spacing=_spacing(nominal),
                       halo=4 if nominal is None else 10, exchange=exchange,
                       params=FilterParams(solve_placement=placement), cull=cull)
    # every rank here is pinned to cuda:0 (LOCAL_WORLD_SIZE unset): the placement check sees it and
    # picks the separate row-guard kernel for the window cull
    assert S.params.window_guard == ("separate" if ws > 1 else "auto")
    if graph == "cycle":   # whole exchange cycles replayed as one hipGraph each
        S.capture_cycle()
    elif graph:
        S.capture()
    S.reset_solves()
    if run == "mixed":   # two single sub-steps, then the rest of that cycle as one partial call
        S.step()
        S.step()
        S.run(steps - 2)
    elif run == "replay":   # the bench's timed path: stats off, then restore() and a stats-on replay
        if graph == "cycle":    # cycle graphs of both statistics settings, as the bench captures them
            S.collect_stats = False
            S.capture_cycle()
            S.collect_stats = True
        snap = S.snapshot()
        S.collect_stats = False
        S.run(steps)
        torch.cuda.synchronize()
        S.check_guard()
        first = S.own.clone()
        assert int(S.stats.abs().sum()) == 0
        S.restore(snap)
        S.collect_stats = True
        S.run(steps)
        torch.cuda.synchronize()
        assert torch.equal(first, S.own)
    elif run:    # cycles (whole, or the part left) through cbf_lattice_cycle_sharded (chained sub-steps)
        S.run(steps)
    else:
        for _ in range(steps):
            S.step()
    torch.cuda.synchronize()
    S.check_guard()
    q.put((rank, S.own.cpu().numpy(), S.status.cpu().numpy(), S.u.cpu().numpy(), S.stats_summary()))
    dist.barrier()
    dist.destroy_process_group()


RANDOM = ("random", 1.0, 3)   # the random-walk nominal control (CBF_NOMINAL_RANDOM)


# placement: where the full QP solves run (cbf_params.solve_inline_max).  These small windows pick
# "inline" under "auto"; the "queued" cases run the queue kernel and its chained binning into the
# next sub-step's workspace (the path of windows above 131,072 agents).  cull "window": every
# sub-step through the lattice-window cull (cbf_lattice_cycle_sharded_ex, CBF_RUN_WINDOW_CULL).
NB = "neighbour"


@pytest.mark.parametrize("ws,k,graph,run,nominal,exchange,placement,cull", [
    (2, 1, False, False, None, NB, "auto", "cells"), (3, 4, False, False, None, NB, "auto", "cells"),
    (2, 4, True, False, None, NB, "auto", "cells"), (3, 4, False, True, None, NB, "auto", "cells"),
    (2, 2, False, True, None, NB, "auto", "cells"), (2, 4, "cycle", True, None, NB, "auto", "cells"),
    (2, 2, False, True, RANDOM, NB, "auto", "cells"), (3, 4, False, "mixed", None, NB, "auto", "cells"),
    (2, 4, False, "replay", None, NB, "auto", "cells"), (3, 4, "cycle", "replay", None, NB, "auto", "cells"),
    (4, 2, False, True, None, NB, "auto", "cells"), (3, 4, False, True, None, "allgather", "auto", "cells"),
    (3, 4, False, True, None, NB, "queued", "cells"), (2, 2, False, True, RANDOM, NB, "queued", "cells"),
    (3, 4, "cycle", "replay", None, NB, "queued", "cells"), (2, 1, False, False, None, NB, "queued", "cells"),
    (2, 1, False, False, None, NB, "auto", "window"), (3, 4, False, True, None, NB, "auto", "window"),
    (2, 4, True, False, None, NB, "auto", "window"), (3, 4, "cycle", "replay", None, NB, "auto", "window"),
    (3, 4, False, "mixed", None, NB, "queued", "window"), (2, 2, False, True, RANDOM, NB, "auto", "window"),
    (4, 2, False, True, None, NB, "queued", "window")])
def test_sharded_equals_single_gpu(ws, k, graph, run, nominal, exchange, placement, cull):
    from cbf_amd import scenarios, swarm
    W, R, steps = 96, 40, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, W, R, steps, q, k, graph, run, nominal, exchange,
                                               placement, cull)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(ws)], key=lambda t: t[0])
    assert not any(isinstance(r[1], str) for r in res), res
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    H = R * ws
    # the oracle's rollout of the whole lattice (test infrastructure, oracle/)
    from oracle import coracle, pyoracle as po
    pos = scenarios.lattice(W, H, seed=7, spacing=_spacing(nominal))
    solves = optimal = relaxed = 0
    for _ in range(steps):
        vel = coracle.consensus_lattice(W, H, 0, H, pos, scenarios.LATTICE_GAIN) if nominal is None else \
            po.random_nominal(pos, 0, nominal[1], nominal[2])
        out = coracle.filter_swarm(po.Params(15), pos, vel, 0)
        pos = coracle.euler(pos, out["u"], scenarios.T)
        solves += int((out["cnt"] > 0).sum())
        optimal += int(((out["status"] & 0xFF) == 1).sum())
        relaxed += int(((out["status"] & 0xFF) == 2).sum())
    assert np.array_equal(np.concatenate([r[1] for r in res]), pos)
    assert np.array_equal(np.concatenate([r[2] for r in res]), out["status"])
    assert np.array_equal(np.concatenate([r[3] for r in res]), out["u"])
    assert sum(r[4]["solves"] for r in res) == solves
    assert sum(r[4]["optimal"] for r in res) == optimal and sum(r[4]["relaxed"] for r in res) == relaxed
    # and the single-GPU fused step of the whole lattice
    L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=7, spacing=_spacing(nominal)), W, H, nominal=nominal,
                           params=swarm.FilterParams(solve_placement=placement))
    for _ in range(steps):
        L.step()
    torch.cuda.synchronize()
    assert np.array_equal(L.pos.cpu().numpy(), pos)


def _worker_breach(rank, ws, port, q):
    import datetime
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    # a rank that stops at a breach leaves its peer in the next collective: a short timeout ends it
    dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=20))
    from cbf_amd.shard import ShardedLattice
    S = ShardedLattice(48, 16, seed=3, halo=2, substeps=1)   # halo 2 is too small for spacing 0.145
    done = 0
    try:
        for _ in range(40):
            S.step()
            done += 1
            torch.cuda.synchronize()   # let the guard read-back of each exchange land
        q.put((rank, "not caught", done))
    except RuntimeError as e:
        q.put((rank, "raised" if "halo guard" in str(e) else "peer stopped", done))


def test_halo_breach_stops_the_rollout_early():
    """A halo that is too small is caught at an exchange during the rollout (the guard flag is read
    back after every exchange), not only by check_guard() at the end."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_breach, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(timeout=120)
    assert any(r[1] == "raised" and r[2] < 5 for r in res), res


# ---- ShardedGroupSwarm (any swarm): entity ranges + one position all-gather per step ----------

def _grid_swarm(W=120, H=100):
    """A 12,000-agent jittered lattice driven by a 4-neighbour Laplacian given as a generic group
    (so the filter takes the cell-list path of filter_swarm, n > 8192)."""
    from cbf_amd import scenarios
    pos = scenarios.lattice(W, H, seed=4)
    rows = []
    for i in range(W * H):
        r, c = divmod(i, W)
        rows.append([j for j in (i - W if r > 0 else -1, i - 1 if c > 0 else -1, i + 1 if c < W - 1 else -1,
                                 i + W if r < H - 1 else -1) if j >= 0])
    return pos, 0, [(0, W * H, rows, None, None, scenarios.LATTICE_GAIN)]


def _group_case(name):
    from cbf_amd import scenarios
    return scenarios.meet_at_center(100) if name == "mac100" else _grid_swarm()


def _group_worker(rank, ws, port, name, steps, q):
    try:
        import datetime
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=60))
        from cbf_amd.shard import ShardedGroupSwarm
        pos0, n_obs, groups = _group_case(name)
        S = ShardedGroupSwarm(pos0, n_obs, groups)
        S.run(steps)
        torch.cuda.synchronize()
        q.put((rank, S.pos.cpu().numpy(), S.u.cpu().numpy(), S.status.cpu().numpy(), S.solves_total()))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        q.put((rank, "error", repr(e)))
        raise


@pytest.mark.parametrize("name,ws,steps", [("mac100", 2, 20), ("grid12k", 2, 4), ("grid12k", 3, 3)])
def test_sharded_group_swarm_equals_single_gpu(name, ws, steps):
    """The any-swarm sharded path on the HIP backend (2 / 3 ranks on one GPU, gloo) == the
    single-GPU GroupSwarm rollout bit for bit on every rank (all-pairs for mac100, the cell list for
    the 12 k swarm), and == the oracle's rollout for mac100."""
    from cbf_amd import swarm
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, ws, port, name, steps, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(ws)], key=lambda t: t[0])
    assert not any(isinstance(r[1], str) for r in res), res
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pos0, n_obs, groups = _group_case(name)
    G = swarm.GroupSwarm(pos0, n_obs, groups)
    solves = 0
    for _ in range(steps):
        out = G.step()
        solves += int((out["nbr_count"] > 0).sum())
    torch.cuda.synchronize()
    ref = G.pos.cpu().numpy()
    for r in res:
        assert np.array_equal(r[1], ref)
    assert np.array_equal(np.concatenate([r[2] for r in res]), out["u_all"].cpu().numpy())
    assert np.array_equal(np.concatenate([r[3] for r in res])[n_obs:], out["status"].cpu().numpy())
    assert sum(r[4] for r in res) == solves
    if name == "mac100":
        from oracle import coracle, pyoracle as po
        pos = pos0.copy()
        for _ in range(steps):
            vel = np.zeros_like(pos)
            for (b, e, rows, anc, rot, scale) in groups:
                rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
                col = np.array([j for r in rows for j in r], np.int32)
                vel[b:e] = coracle.consensus_csr(pos[b:e], rp, col, 0, e - b, anchors=anc, rot=rot, scale=scale)
            o = coracle.filter_swarm(po.Params(15), pos, vel, n_obs)
            u = vel.copy()
            u[n_obs:] = o["u"]
            pos = coracle.euler(pos, u, 1 / 30)
        assert np.array_equal(ref, pos)
