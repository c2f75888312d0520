"""GPU box: relaxation-count and neighbour-count histograms of the HOCBF lattice step over a run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cbf_amd import scenarios, swarm  # noqa: E402

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
for step in range(121):
    L.step()
    if step % 30 == 0:
        torch.cuda.synchronize()
        st = L.status.cpu().numpy()
        it = st >> 8
        cnt = L.nbr_count.cpu().numpy()
        print(step, "iters hist", np.bincount(np.minimum(it, 20)).tolist(), "nbr hist",
              np.bincount(np.minimum(cnt, 24)).tolist(), flush=True)
