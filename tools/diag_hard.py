"""GPU box: size of the lattice step's hard-QP queue (QPs not solved at the origin) over a run."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cbf_amd import scenarios, swarm

def a256(b):
    return (b + 255) // 256 * 256

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN)
n = W * H
nc = L.grid.nx * L.grid.ny
ntiles = (nc + 2047) // 2048
off = a256(4 * nc) + a256(4 * (nc + 1)) + a256(8 * ntiles) + 256 + a256(16 * n) + 2 * a256(16 * n) + a256(4 * n) + a256(16 * n) + a256(8 * n)
for step in range(240):
    L.step()
    if step % 20 == 0 or step == 239:
        torch.cuda.synchronize()
        hq = int(L.ws[off:off + 4].view(torch.int32).item())
        st = L.status.cpu().numpy()
        print(step, "hard queue", hq, "frac", hq / n, "relaxed", float(((st & 0xFF) == 2).mean()),
              "iters max", int((st >> 8).max()), flush=True)
