"""GPU box (diagnostic): which egos of the cfg4 window cull take the unbounded walk, and how long
are their walks?  Runs the 1024 x 1024 lattice with the window cull and, at timesteps 5..25 (the
driver's span), restates the tile's walk rule on the host from that timestep's input positions:
row window from the row guard (fp64 extents here; the filter's fp32 words are at most one ulp
looser), sentinels at c -+ 2, then c -+ 3, per row of the window.  For each walking ego it prints
the per-row walk lengths (columns beyond c -+ 3 to the first holding sentinel), its place in the
tile grid, and how many 16-column blocks of each row overlap [x - d, x + d] (what a block-extent
walk would visit).  Usage: python tools/diag_walks.py [spacing] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cbf_amd import scenarios, swarm

spacing = float(sys.argv[1]) if len(sys.argv) > 1 else 0.145
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 26
W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0, spacing=spacing), W, H, gain=scenarios.LATTICE_GAIN,
                       cull="window")
L.collect_stats = False
d = 0.2
while d * d < 0.04:
    d = np.nextafter(d, np.inf)
tot = 0
lens = []
for t in range(steps):
    pos = L.pos.cpu().numpy().reshape(H, W, 2)
    if t >= 5:
        x, y = pos[:, :, 0], pos[:, :, 1]
        fin = np.isfinite(pos).all(axis=2)
        xf = np.where(fin, x, np.inf)
        xg = np.where(fin, x, -np.inf)
        rs = np.minimum.accumulate(xf[:, ::-1], axis=1)[:, ::-1]   # min over columns >= c
        rp = np.maximum.accumulate(xg, axis=1)                     # max over columns <= c
        lo = np.where(fin, y, np.inf).min(axis=1)
        hi = np.where(fin, y, -np.inf).max(axis=1)
        sylo = np.minimum.accumulate(lo[::-1])[::-1]
        pyhi = np.maximum.accumulate(hi)
        unsorted = [int(r) for r in range(H) if not (fin[r].all() and (np.diff(x[r]) >= 0).all())]
        walkers = []
        for r in range(H):
            rows = range(max(0, r - 8), min(H, r + 9))
            c = np.arange(W)
            slow = np.zeros(W, bool)
            for rr in rows:
                dr = rr - r
                # per ego: is row rr in its window?
                if dr > 0:    # sylo is non-decreasing, so row rr is in the window iff its own bound fails
                    inwin = ~(sylo[rr] - y[r] > d)
                elif dr < 0:
                    inwin = ~(y[r] - pyhi[rr] > d)
                else:
                    inwin = np.ones(W, bool)
                if dr != 0 and abs(dr) > 3:
                    slow |= inwin & fin[r]
                    continue
                sR2 = np.where(c + 2 < W, rs[rr, np.minimum(c + 2, W - 1)], np.inf)
                sL2 = np.where(c - 2 >= 0, rp[rr, np.maximum(c - 2, 0)], -np.inf)
                sR3 = np.where(c + 3 < W, rs[rr, np.minimum(c + 3, W - 1)], np.inf)
                sL3 = np.where(c - 3 >= 0, rp[rr, np.maximum(c - 3, 0)], -np.inf)
                needR = ~(sR2 - x[r] > d)
                needL = ~(x[r] - sL2 > d)
                slow |= inwin & fin[r] & ((needR & ~(sR3 - x[r] > d)) | (needL & ~(x[r] - sL3 > d)))
            for cc in np.nonzero(slow)[0]:
                walkers.append((r, int(cc)))
        tot += len(walkers)
        desc = []
        for (r, cc) in walkers[:8]:
            xe, ye = x[r, cc], y[r, cc]
            per = []
            for rr in range(max(0, r - 3), min(H, r + 4)):
                if rr > r and sylo[rr] - ye > d:
                    continue
                if rr < r and ye - pyhi[rr] > d:
                    continue
                right = next((k for k in range(cc + 1, W) if rs[rr, k] - xe > d), W) - cc - 1
                left = cc - next((k for k in range(cc - 1, -1, -1) if xe - rp[rr, k] > d), -1) - 1
                bl = 0
                for b in range(0, W, 16):
                    seg = x[rr, b:b + 16][fin[rr, b:b + 16]]
                    if seg.size and not (seg.min() - xe > d) and not (xe - seg.max() > d):
                        bl += 1
                per.append((rr - r, right, left, bl))
                lens.append(right + left)
            desc.append(f"ego ({r},{cc}) tile ({r // 8},{cc // 64}) rows(dr,R,L,blocks)={per}")
        print(f"timestep {t}: {len(walkers)} walkers; unsorted rows {unsorted[:10]}{'...' if len(unsorted) > 10 else ''} "
              f"({len(unsorted)})", flush=True)
        for s in desc:
            print("   ", s, flush=True)
    L.step()
torch.cuda.synchronize()
print(f"total walkers {tot}; walk columns per row: mean {np.mean(lens) if lens else 0:.1f}, "
      f"max {max(lens) if lens else 0}", flush=True)
