"""Diagnostic: is the sharded lattice step host-bound?  One rank (RCCL, world size 1), 128 rows,
8 sub-steps per exchange, the bench's cycle graph; times the host's enqueue of each part of an
exchange cycle (no synchronisation inside the loop) against the wall time of the whole rollout.
Usage: python tools/diag_shard_host.py [rows] [cycles]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
    from cbf_amd.shard import ShardedLattice
    S = ShardedLattice(1024, rows, seed=0, halo=4, substeps=8)
    S.collect_stats = False
    S.capture_cycle()
    S.run(16)
    torch.cuda.synchronize()
    parts = {"poll": 0.0, "pack": 0.0, "collective": 0.0, "unpack": 0.0, "readback": 0.0, "replay": 0.0}
    g = S.cycle_graphs[False]
    t0 = time.perf_counter()
    for _ in range(cycles):
        a = time.perf_counter()
        S.be.poll_guard()
        b = time.perf_counter()
        S.be.pack(S)
        c = time.perf_counter()
        S._collective()
        d = time.perf_counter()
        S.be.unpack_guard(S)
        e = time.perf_counter()
        S.be.arm_guard_readback()
        f = time.perf_counter()
        g.replay()
        h = time.perf_counter()
        for k, v in zip(parts, (b - a, c - b, d - c, e - d, f - e, h - f)):
            parts[k] += v
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    us = {k: round(v / cycles * 1e6, 1) for k, v in parts.items()}
    print(f"rows {rows}: per 8-step cycle host enqueue {host / cycles * 1e6:.1f} us {us}, wall {wall / cycles * 1e6:.1f} us "
          f"({wall / cycles / 8 * 1e6:.1f} us/step)")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
