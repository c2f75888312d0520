"""Which QPs leave the filter for the exact solve, and how many +1 relaxations they take: the
cfg4 lattice (spacing 0.145) under the window cull at 1024 and 128 rows, status histograms of
timesteps 6..25, and the positions before timestep 7 with that step's status (npz under
gpurun_out/hardqp/) for offline analysis with the oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

out = "gpurun_out/hardqp"
os.makedirs(out, exist_ok=True)
for H in (1024, 128):
    L = swarm.LatticeSwarm(scenarios.lattice(1024, H, seed=0, spacing=0.145), 1024, H, gain=0.25, cull="window")
    L.collect_stats = False
    L.run(6)
    pos6 = L.pos.cpu().numpy().copy()
    L.run(19, history=True)
    _, _, st, cnt = L.history(19)
    st = st.cpu().numpy()
    code, it = st & 0xFF, st >> 8
    print(f"H={H}: codes {dict(zip(*np.unique(code, return_counts=True)))}")
    r = it[it > 0]
    print(f"  relaxed egos per step {r.size / 19:.1f}; iters histogram "
          f"{dict(zip(*np.unique(np.minimum(r, 40), return_counts=True)))}")
    np.savez_compressed(f"{out}/h{H}.npz", pos6=pos6, status7=st[0], cnt7=cnt[0].cpu().numpy())
