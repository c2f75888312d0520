"""GPU box (diagnostic): how long are the window cull's unbounded walks at cfg4?  Runs the 1024 x 1024
lattice with the window cull for 25 timesteps (the driver's span is 6-25) and, from each
timestep's input positions, restates the row guard on the host (fp64 row extents, suffix minimum /
prefix maximum; the filter uses the same values rounded outward to fp32) to list the egos whose
row window leaves the staged +-3 rows, with their row-window sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from cbf_amd import scenarios, swarm

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN, cull="window")
L.collect_stats = False
d = 0.2
while d * d < 0.04:
    d = np.nextafter(d, np.inf)
for t in range(26):
    pos = L.pos.cpu().numpy().reshape(H, W, 2)
    if t >= 5:
        y = pos[:, :, 1]
        fin = np.isfinite(pos).all(axis=2)
        lo = np.where(fin, y, np.inf).min(axis=1)
        hi = np.where(fin, y, -np.inf).max(axis=1)
        sylo = np.minimum.accumulate(lo[::-1])[::-1]   # min over rows >= r
        pyhi = np.maximum.accumulate(hi)                 # max over rows <= r
        ku = np.zeros((H, W), np.int64)
        kd = np.zeros((H, W), np.int64)
        for k in range(1, 64):
            up = np.zeros((H, W), bool)
            up[:H - k] = ~(sylo[k:, None] - y[:H - k] > d)
            dn = np.zeros((H, W), bool)
            dn[k:] = ~(y[k:] - pyhi[:H - k, None] > d)
            ku += up & (ku == k - 1)
            kd += dn & (kd == k - 1)
        walk = (ku > 3) | (kd > 3)
        n = int(walk.sum())
        rows = (ku + kd + 1)[walk]
        print(f"timestep {t}: {n} egos with a row window beyond +-3 rows; window rows {sorted(rows.tolist())[:12]}"
              f"{' ...' if n > 12 else ''}; where {[tuple(map(int, a)) for a in np.argwhere(walk)[:6]]}", flush=True)
    L.step()
torch.cuda.synchronize()
