"""A/B on the GPU box: cfg4 run(10) graphs with and without the rollout statistics (collect_stats,
stats=NULL), interleaved, plus a bit-identity check of the two trajectories, for the package in
<tree-root>.  Usage: python tools/ab_stats.py <tree-root> [spacing]"""
import json
import sys
import time

root = sys.argv[1] if len(sys.argv) > 1 else "."
spacing = float(sys.argv[2]) if len(sys.argv) > 2 else 0.145
sys.path.insert(0, root)
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402


def timed(S, steps=200, chunk=10):
    S.run(chunk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // chunk):
        S.run(chunk)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / steps * 1e6, 2)


def main():
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0, spacing=spacing)
    A = swarm.LatticeSwarm(pos, W, H)
    B = swarm.LatticeSwarm(pos, W, H)
    B.collect_stats = False
    for S in (A, B):
        S.capture(steps=10)
    for S in (A, B):
        S.run(10)
    torch.cuda.synchronize()
    same = bool(torch.equal(A.pos, B.pos)) and bool(torch.equal(A.u, B.u)) and bool(torch.equal(A.status, B.status))
    res = {"tree": root, "spacing": spacing, "bit_identical": same, "stats_us": [], "nostats_us": []}
    for _ in range(3):
        res["stats_us"].append(timed(A))
        res["nostats_us"].append(timed(B))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
