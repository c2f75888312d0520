"""GPU box: size of the lattice step's hard-QP queue over a run.

An ego solved at the origin returns u = clip(u0); the hard queue holds the egos whose QP needed
the full solve, i.e. (filter ran) and u != clip(u0).  Prints the count every 20 steps.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cbf_amd import scenarios, swarm

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN)
n = W * H
ms = 15.0
for step in range(int(os.environ.get("DIAG_STEPS", "240"))):
    L.step()
    if step % 20 == 0:
        torch.cuda.synchronize()
        ran = L.nbr_count.view(-1) > 0
        u0 = L.vel.view(-1, 2).clamp(-ms, ms)
        hard = ran & (L.u.view(-1, 2) != u0).any(dim=1)
        st = L.status.view(-1)
        print(step, "hard", int(hard.sum()), "frac %.5f" % (float(hard.sum()) / n),
              "relaxed %.4f" % float(((st & 0xFF) == 2).float().mean()),
              "iters max", int((st >> 8).max()), "nbrs mean %.2f max %d" % (float(L.nbr_count.float().mean()),
                                                                             int(L.nbr_count.max())), flush=True)
