"""A/B on the GPU box: cfg4 run(10) graphs with and without the rollout statistics (stats=NULL),
interleaved, plus a bit-identity check of the two trajectories.  python tools/ab_stats.py"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from cbf_amd import _lib, scenarios, swarm  # noqa: E402
from cbf_amd._lib import lib, ptr, check, stream_handle  # noqa: E402


class NoStats(swarm.LatticeSwarm):
    def _launch_run(self, steps):
        check(lib.cbf_lattice_run(self.cp, _lib.C.byref(self.grid), self.W, self.H, ptr(self.pos), self.gain, self.T,
                                  steps, ptr(self.vel), ptr(self.u), ptr(self.status), ptr(self.nbr_count),
                                  None, ptr(self.ws), self.ws_bytes, stream_handle()), "cbf_lattice_run")


def timed(S, steps=200, chunk=10):
    S.run(chunk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // chunk):
        S.run(chunk)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0, spacing=0.145)
    A = swarm.LatticeSwarm(pos, W, H)
    B = NoStats(pos, W, H)
    for S in (A, B):
        S.capture(steps=10)
    # identical trajectories (same warm-up count: capture ran one un-captured call each)
    for S in (A, B):
        S.run(10)
    torch.cuda.synchronize()
    same = bool(torch.equal(A.pos, B.pos)) and bool(torch.equal(A.u, B.u)) and bool(torch.equal(A.status, B.status))
    res = {"bit_identical": same, "stats_us": [], "nostats_us": []}
    for _ in range(3):
        res["stats_us"].append(timed(A))
        res["nostats_us"].append(timed(B))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
