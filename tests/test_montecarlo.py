"""Scenario sharding of the batched Monte-Carlo rollout (cbf_amd/montecarlo.py) on
CPU with the gloo backend at world size 2 and 3.  The device work is done by an oracle backend
(test infrastructure), so this checks the sharding and the end-of-run reductions: the combined
totals of the ranks must equal those of one unsharded oracle rollout of the whole batch."""
import math
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from cbf_amd import scenarios
from cbf_amd.montecarlo import MonteCarlo, shard_bounds
from oracle import coracle, pyoracle as po

N_SCEN, N_O, N_A, STEPS, CHUNKS = 23, 6, 5, 12, 3


class OracleBackend:
    def __init__(self):
        self.p = po.Params(15)

    def tensor(self, a):
        return np.array(a, dtype=np.float64)

    def rollout(self, pos, n_o, n_a, steps, ga):
        th = -math.pi / n_o
        new, cnt, mv, sf = coracle.mc_rollout(self.p, pos, n_o, n_a, steps, 1 / 30, (math.cos(th), math.sin(th)),
                                              1.0, ga, safety=True)
        pos[...] = new
        return cnt, mv, sf


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    mc = MonteCarlo(N_SCEN, N_O, N_A, seed=3, ga=1.0, backend=OracleBackend())
    for _ in range(CHUNKS):
        mc.run(STEPS)
    q.put((rank, mc.lo, mc.hi, mc.pos.copy(), mc.totals()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover_the_batch():
    for n in (1, 7, 100_000):
        for ws in (1, 2, 3, 8):
            b = [shard_bounds(n, ws, r) for r in range(ws)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(ws - 1))


@pytest.mark.parametrize("ws", [2, 3])
def test_scenario_sharded_totals_equal_unsharded(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # one unsharded rollout of the whole batch
    pos = scenarios.mc_scenarios(N_SCEN, N_O, N_A, seed=3)
    be = OracleBackend()
    cnt = np.zeros(4, np.int64)
    mv = vo = 0.0
    d2 = np.inf
    for _ in range(CHUNKS):
        c, m, s = be.rollout(pos, N_O, N_A, STEPS, 1.0)
        cnt += c.sum(0)
        mv = max(mv, m.max())
        vo = max(vo, s[:, 0].max())
        d2 = min(d2, s[:, 1].min())
    assert np.array_equal(np.concatenate([r[3] for r in res]), pos)
    for _, lo, hi, _, tot in res:     # every rank reports the same, whole-batch totals
        assert (tot["calls"], tot["relaxed"], tot["box_infeasible"], tot["relax_cap"]) == tuple(int(v) for v in cnt)
        assert tot["max_violation_optimal"] == mv and tot["max_violation_original_rows_relaxed"] == vo
        assert tot["min_pairwise_distance"] == math.sqrt(d2)
    assert sum(r[2] - r[1] for r in res) == N_SCEN
