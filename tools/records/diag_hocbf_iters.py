"""GPU box: relaxation-count and neighbour-count histograms of the HOCBF lattice step (cfg4 shape)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cbf_amd import scenarios, swarm

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
for step in range(60):
    L.step()
    if step in (0, 20, 59):
        torch.cuda.synchronize()
        st = L.status.cpu().numpy()
        cnt = L.nbr_count.cpu().numpy()
        it = st >> 8
        code = st & 0xFF
        print(step, "codes", np.bincount(code, minlength=6).tolist(), "iters", np.bincount(it, minlength=4)[:12].tolist(),
              "nbrs", np.bincount(cnt, minlength=10)[:16].tolist(), flush=True)
