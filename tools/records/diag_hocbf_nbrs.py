"""GPU box: neighbour-count and relaxation-count histograms of the HOCBF lattice step at the cfg4
shape over the bench's span (20 warm-up + 100 timed steps), for sizing the main kernel's LDS rows
(egos with more rows than it holds go to k_lattice_filter_hocbf_wide)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from cbf_amd import scenarios, swarm

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
for step in range(120):
    L.step()
    if step in (0, 19, 59, 119):
        torch.cuda.synchronize()
        st = L.status.cpu().numpy()
        cnt = L.nbr_count.cpu().numpy()
        h = np.bincount(cnt, minlength=12)
        print(step, "iters", np.bincount(st >> 8, minlength=3)[:6].tolist(), "nbrs", h[:12].tolist(),
              "m>5 %.4f m>6 %.4f m>8 %.4f" % ((cnt > 5).mean(), (cnt > 6).mean(), (cnt > 8).mean()), flush=True)
