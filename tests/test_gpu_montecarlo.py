"""The cfg5 scenario split (cbf_amd/montecarlo.py; meet_at_center.py:76-153 per
scenario) through the HIP backend at gloo world size 2 and 3 on one GPU: spawned ranks, each rolling
out its contiguous scenario range with cbf_mc_rollout on cuda:0 and combining the totals by the
all-reduces of MonteCarlo.totals().  The ranks' positions, concatenated, and their whole-batch totals
must equal one unsharded HIP rollout bit for bit, and the oracle's rollout of a sample of the
scenarios (the same counters and positions).  (The nccl branch of totals() needs one GPU per rank:
the driver's multi-GPU node.)"""
import math
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU boxes but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from cbf_amd import scenarios  # noqa: E402
from cbf_amd.montecarlo import MonteCarlo  # noqa: E402
from oracle import coracle, pyoracle as po  # noqa: E402

N_SCEN, N_O, N_A, STEPS, CHUNKS, SEED, GA = 301, 8, 8, 10, 3, 5, 1.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        mc = MonteCarlo(N_SCEN, N_O, N_A, seed=SEED, ga=GA)  # HipBackend
        for _ in range(CHUNKS):
            mc.run(STEPS)
        tot = mc.totals()
        q.put((rank, mc.lo, mc.hi, mc.pos.cpu().numpy(), tot))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent, which fails the test with it
        q.put((rank, None, None, None, repr(e)))
        raise


def _unsharded():
    mc = MonteCarlo(N_SCEN, N_O, N_A, seed=SEED, ga=GA)
    for _ in range(CHUNKS):
        mc.run(STEPS)
    return mc.pos.cpu().numpy(), mc.totals()


@pytest.mark.parametrize("ws", [2, 3])
def test_hip_scenario_split_equals_unsharded_and_oracle(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(ws)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] is not None, f"rank {r[0]} failed: {r[4]}"
    assert all(p.exitcode == 0 for p in procs)
    pos, tot = _unsharded()
    assert sum(r[2] - r[1] for r in res) == N_SCEN
    assert np.array_equal(np.concatenate([r[3] for r in res]), pos)
    for r in res:  # every rank reports the whole batch's totals
        assert r[4] == tot, (r[0], r[4], tot)
    assert tot["calls"] > 0 and tot["relaxed"] > 0
    # the oracle on a sample of the scenarios (a contiguous run across the ranks' boundaries)
    lo, hi = N_SCEN // ws - 3, N_SCEN // ws + 4
    ref = scenarios.mc_scenarios(N_SCEN, N_O, N_A, seed=SEED)[lo:hi]
    p, th = po.Params(15), -math.pi / N_O
    for _ in range(CHUNKS):
        ref, cnt, mv = coracle.mc_rollout(p, ref, N_O, N_A, STEPS, 1 / 30, (math.cos(th), math.sin(th)), 1.0, GA)
    assert np.array_equal(pos[lo:hi], ref)
