"""Row-stripe sharding (cbf_amd/shard.py) on CPU with the gloo backend, world_size 2 and 3.
The device work is done by an oracle backend (test infrastructure), so this checks the
exchange / window / guard logic: the sharded rollout must equal the single-lattice oracle
rollout bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cbf_amd import scenarios
from cbf_amd.shard import ShardedLattice, guard_ok, sub_extents
from oracle import coracle, pyoracle as po


IDENT = np.array([np.inf, -np.inf, -np.inf, np.inf, np.inf, -np.inf])


class OracleBackend:
    """Device work restated on the CPU (oracle): the same pack / unpack+guard / sub-step contract
    as HipBackend, including the guard running at the exchange after the sub-steps it certifies."""

    def __init__(self, W, H, gain, T, radius, nsub):
        self.W, self.H, self.gain, self.T, self.radius, self.nsub = W, H, gain, T, radius, nsub
        self.p = po.Params(15)
        self.flag = 0
        self.recs = np.tile(IDENT, (nsub, 1))

    def tensor(self, a):
        return torch.as_tensor(np.ascontiguousarray(a)).clone()

    def pack(self, S):
        rs = S.G * S.W * 2
        own = S.own.reshape(-1)
        if S.exchange_mode == "neighbour":    # chunk q: [records | first rows to q = r-1, last rows to r+1]
            for q in range(S.ws):
                o = S.chunk_offset(q)
                for s in range(self.nsub):
                    S.send[o + 8 * s:o + 8 * s + 6].copy_(torch.as_tensor(self.recs[s]))
                r8 = o + 8 * self.nsub
                if q == S.rank - 1:
                    S.send[r8:r8 + rs].copy_(own[:rs])
                elif q == S.rank + 1:
                    S.send[r8:r8 + rs].copy_(own[own.numel() - rs:])
        else:
            S.send[:rs].copy_(own[:rs])
            S.send[rs:2 * rs].copy_(own[own.numel() - rs:])
            for s in range(self.nsub):
                S.send[S.slab + 8 * s:S.slab + 8 * s + 6].copy_(torch.as_tensor(self.recs[s]))
        self.recs = np.tile(IDENT, (self.nsub, 1))

    def unpack_guard(self, S):
        W, rs = S.W, S.G * S.W * 2
        nbr = S.exchange_mode == "neighbour"
        r8 = 8 * self.nsub
        wv = S.wpos.view(-1)
        if S.rank > 0:
            lo = S.chunk_offset(S.rank - 1) + r8 if nbr else (S.rank - 1) * S.stride + rs
            n = (S.rb - S.w0) * W * 2
            wv[:n].copy_(S.recv[lo + rs - n:lo + rs])
        if S.rank < S.ws - 1:
            hi = S.chunk_offset(S.rank + 1) + r8 if nbr else (S.rank + 1) * S.stride
            a = (S.re - S.w0) * W * 2
            n = (S.w1 - S.re) * W * 2
            wv[a:a + n].copy_(S.recv[hi:hi + n])
        for s in range(self.nsub):
            base = [S.chunk_offset(q) if nbr else q * S.stride + S.slab for q in range(S.ws)]
            recs = np.stack([S.recv[b + 8 * s:b + 8 * s + 6].numpy() for b in base])
            if not guard_ok(recs, S.rank, self.radius):
                self.flag = 1

    def lattice_step(self, S, s, sub):
        W, H = self.W, self.H
        win = S.wpos.numpy()[(sub.w0 - S.w0) * W:(sub.w1 - S.w0) * W]
        self.recs[s] = sub_extents(win, W, sub.w0, sub.a, sub.b, S.rb, S.re, sub.guard)
        full = np.zeros((W * H, 2))
        full[sub.w0 * W:sub.w1 * W] = win
        lo = sub.w0 if sub.w0 == 0 else sub.w0 + 1        # rows whose nominal control exists
        hi = sub.w1 if sub.w1 == H else sub.w1 - 1
        vel = coracle.consensus_lattice(W, H, lo, hi, full, self.gain)
        cand = full[lo * W:hi * W]
        eb, ee = (sub.a - lo) * W, (sub.b - lo) * W
        out = coracle.filter_swarm(self.p, cand, vel, 0, eb, ee)
        new = coracle.euler(cand[eb:ee], out["u"], self.T)
        o = (sub.a - S.w0) * W
        n = (sub.b - sub.a) * W
        S.wpos[o:o + n].copy_(torch.as_tensor(new))
        S.wvel[o:o + n].copy_(torch.as_tensor(vel[eb:ee])); S.wu[o:o + n].copy_(torch.as_tensor(out["u"]))
        S.wstatus[o:o + n].copy_(torch.as_tensor(out["status"])); S.wcnt[o:o + n].copy_(torch.as_tensor(out["cnt"]))
        oe, of = (S.rb - sub.a) * W, (S.re - sub.a) * W
        S.stats[0] += int((out["cnt"][oe:of] > 0).sum())

    def arm_guard_readback(self):
        pass

    def poll_guard(self):
        return bool(self.flag)

    def guard_failed(self):
        return bool(self.flag)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, ws, port, W, R, steps, halo, q, k=1, exchange="neighbour"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    H = R * ws
    be = OracleBackend(W, H, scenarios.LATTICE_GAIN, scenarios.T, 0.2, k)
    S = ShardedLattice(W, R, seed=2, halo=halo, substeps=k, backend=be, exchange=exchange)
    for _ in range(steps):
        S.step()
    S.check_guard()
    q.put((rank, S.own.numpy().copy(), S.u.numpy().copy(), S.status.numpy().copy(), int(S.stats[0])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,k,exchange", [(2, 1, "neighbour"), (3, 1, "neighbour"), (2, 2, "neighbour"),
                                           (3, 3, "neighbour"), (4, 2, "neighbour"), (3, 2, "allgather")])
def test_sharded_rollout_equals_single_lattice(ws, k, exchange):
    W, R, steps, halo = 20, 12, 5, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, W, R, steps, halo, q, k, exchange)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H = R * ws
    pos = scenarios.lattice(W, H, seed=2)
    p = po.Params(15)
    solves = 0
    for _ in range(steps):
        vel = coracle.consensus_lattice(W, H, 0, H, pos, scenarios.LATTICE_GAIN)
        out = coracle.filter_swarm(p, pos, vel, 0)
        solves += int((out["cnt"] > 0).sum())
        pos = coracle.euler(pos, out["u"], scenarios.T)
    got = np.concatenate([r[1] for r in res])
    assert np.array_equal(got, pos)
    assert np.array_equal(np.concatenate([r[2] for r in res]), out["u"])
    assert np.array_equal(np.concatenate([r[3] for r in res]), out["status"])
    assert sum(r[4] for r in res) == solves


def test_neighbour_splits_send_rows_to_neighbours_only():
    """Chunk sizes of the neighbour exchange (cbf_halo_nbr_elems / nbr_chunk_off in swarm.hip):
    records to every rank, rows only to rank +- 1, and a symmetric send / receive pattern."""
    ws, rows, k = 5, 100, 3
    for r in range(ws):
        sp = ShardedLattice.nbr_splits(ws, r, rows, k)
        assert [q for q in range(ws) if sp[q] > 8 * k] == [q for q in (r - 1, r + 1) if 0 <= q < ws]
        # what rank r receives from q is what q sends to r
        assert sp == [ShardedLattice.nbr_splits(ws, q, rows, k)[r] for q in range(ws)]


def test_guard_logic():
    W, halo = 10, 4
    a = scenarios.LATTICE_SPACING
    pos = scenarios.lattice(W, 30, seed=0)
    recs = np.stack([sub_extents(pos, W, 0, 10 * r, 10 * r + 10, 10 * r, 10 * r + 10, halo - 1) for r in range(3)])
    for r in range(3):
        assert guard_ok(recs, r, 0.2)
    bad = recs.copy()
    bad[0, 2] = recs[1, 0] - 0.1            # rank 0's rows outside the band reach into rank 1's range
    assert not guard_ok(bad, 1, 0.2)
    assert guard_ok(bad, 2, 0.2)
    bad = recs.copy()
    bad[2, 4] = recs[0, 1] + 0.05           # rank 2 reaches down to rank 0
    assert not guard_ok(bad, 0, 0.2)
    ident = np.array([np.inf, -np.inf, -np.inf, np.inf, np.inf, -np.inf])
    assert guard_ok(np.stack([ident, recs[1], ident]), 1, 0.2)    # unrecorded sub-steps pass
    assert a * (halo - 2) > 0.2            # default halo leaves slack for the jittered lattice


def _worker_small_halo(rank, ws, port, q, k, exchange):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    W, R = 12, 6
    be = OracleBackend(W, R * ws, scenarios.LATTICE_GAIN, scenarios.T, 0.2, k)
    S = ShardedLattice(W, R, seed=3, halo=2, substeps=k, backend=be, exchange=exchange)
    for _ in range(k):
        S.step()
    try:
        S.check_guard()
        q.put((rank, "ok"))
    except RuntimeError:
        q.put((rank, "raised"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("k,exchange", [(1, "neighbour"), (2, "neighbour"), (2, "allgather")])
def test_too_small_halo_is_caught_after_the_step(k, exchange):
    """halo 2 lets rows two apart (0.29 - jitter < 0.2) reach past the candidate rows: the
    guard, run at the exchange after the step, must flag it and check_guard() must raise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_small_halo, args=(r, 2, port, q, k, exchange)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert any(r[1] == "raised" for r in res)


# ---- ShardedGroupSwarm: any swarm, contiguous entity ranges, one all-gather per timestep ------

class OracleGroupBackend:
    """ShardedGroupSwarm's device work restated on the CPU (oracle)."""

    def __init__(self, groups):
        self.p = po.Params(15)
        self.groups = []
        for (b, e, rows, anc, rot, scale) in groups:
            rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
            col = np.array([j for r in rows for j in r], np.int32)
            self.groups.append((b, e, rp, col, anc, rot, scale))

    def tensor(self, a):
        return torch.as_tensor(np.ascontiguousarray(a)).clone()

    def nominal(self, pos, vel):
        p = pos.numpy()
        for (b, e, rp, col, anc, rot, scale) in self.groups:
            vel[b:e].copy_(torch.as_tensor(coracle.consensus_csr(p[b:e], rp, col, 0, e - b, anchors=anc, rot=rot,
                                                                 scale=scale)))

    def filter(self, pos, vel, n_obs, eb, ee):
        out = coracle.filter_swarm(self.p, pos.numpy(), vel.numpy(), n_obs, eb, ee)
        return torch.as_tensor(out["u"]), torch.as_tensor(out["status"]), torch.as_tensor(out["cnt"])

    def euler(self, pos, u, T):
        pos.copy_(torch.as_tensor(coracle.euler(pos.numpy(), u.numpy(), T)))


def _group_case(name):
    if name == "car":
        return scenarios.cross_and_rescue()
    return scenarios.meet_at_center(int(name[3:]))


def _group_worker(rank, ws, port, name, steps, q):
    from cbf_amd.shard import ShardedGroupSwarm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    pos0, n_obs, groups = _group_case(name)
    S = ShardedGroupSwarm(pos0, n_obs, groups, backend=OracleGroupBackend(groups))
    S.run(steps)
    q.put((rank, S.pos.numpy().copy(), S.u.numpy().copy(), S.solves_total()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,ws", [("car", 2), ("mac10", 3), ("mac100", 2), ("mac100", 3)])
def test_sharded_group_swarm_equals_single_domain(name, ws):
    """Any-swarm sharding (entity ranges + one position all-gather per step) == the single-domain
    oracle rollout of the caller loop bit for bit, on every rank; solves summed over ranks."""
    steps = 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, ws, port, name, steps, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, n_obs, groups = _group_case(name)
    be = OracleGroupBackend(groups)
    solves = 0
    for _ in range(steps):
        vel = torch.zeros((len(pos), 2), dtype=torch.float64)
        be.nominal(torch.as_tensor(pos), vel)
        vel = vel.numpy()
        out = coracle.filter_swarm(be.p, pos, vel, n_obs)
        solves += int((out["cnt"] > 0).sum())
        u = vel.copy()
        u[n_obs:] = out["u"]
        pos = coracle.euler(pos, u, scenarios.T)
    for r in res:
        assert np.array_equal(r[1], pos)
    assert np.array_equal(np.concatenate([r[2] for r in res]), u)
    assert sum(r[3] for r in res) == solves


def test_ranks_share_gpu_reads_the_local_world_size(monkeypatch):
    """ShardedLattice takes the window cull's separate row-guard kernel when its node runs more
    ranks than GPUs (LOCAL_WORLD_SIZE from torchrun / bench.py's launcher against the device
    count); FilterParams validates the choice."""
    import torch
    from cbf_amd import shard, swarm
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert shard.ranks_share_gpu(2)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert not shard.ranks_share_gpu(8)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert not shard.ranks_share_gpu(8)
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert not shard.ranks_share_gpu(4) and shard.ranks_share_gpu(16)
    assert swarm.FilterParams(window_guard="separate").c().launch_flags == 1
    assert swarm.FilterParams().c().launch_flags == 0
    import pytest
    with pytest.raises(ValueError):
        swarm.FilterParams(window_guard="later").c()
