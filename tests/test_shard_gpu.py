"""Sharded lattice step on the HIP path: 2 and 3 ranks rehearsed on one GPU (gloo, host-staged
exchange), with 1 and 4 sub-steps per exchange (6 steps: the last cycle is partial), compared
bit-for-bit with the single-GPU step of the whole lattice."""
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


def _worker(rank, ws, port, W, R, steps, q, k=4, graph=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from cbf_amd.shard import ShardedLattice
    S = ShardedLattice(W, R, seed=7, substeps=k)
    if graph:
        S.capture()
    S.reset_solves()
    for _ in range(steps):
        S.step()
    torch.cuda.synchronize()
    S.check_guard()
    q.put((rank, S.own.cpu().numpy(), S.status.cpu().numpy(), S.solves_total()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,k,graph", [(2, 1, False), (3, 4, False), (2, 4, True)])
def test_sharded_equals_single_gpu(ws, k, graph):
    from cbf_amd import scenarios, swarm
    W, R, steps = 96, 40, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, W, R, steps, q, k, graph)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    H = R * ws
    L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=7), W, H)
    L.reset_solves()
    for _ in range(steps):
        L.step()
    torch.cuda.synchronize()
    assert np.array_equal(np.concatenate([r[1] for r in res]), L.pos.cpu().numpy())
    assert np.array_equal(np.concatenate([r[2] for r in res]), L.status.cpu().numpy())
    assert sum(r[3] for r in res) == L.solves_total()
