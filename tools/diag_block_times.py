"""Diagnostic (a tree built with CBF_DIAG_BLOCK_TIMES, tools/mk_ab.sh): start / end times of every
k_window_tile block of one launch at the driver's timesteps (cfg4, 1 M agents), and how many blocks
are resident over the launch -- the tail of its 2.67 rounds.  Usage: python tools/diag_block_times.py <tree>"""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, sys.argv[1])
import torch  # noqa: E402
from cbf_amd import _lib, scenarios, swarm  # noqa: E402

W = H = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0, spacing=float(sys.argv[2]) if len(sys.argv) > 2 else 0.145),
                       W, H, gain=0.25, cull="window")
L.collect_stats = False
f = _lib.lib.cbf_diag_block_times
f.argtypes = [C.c_void_p, C.c_int]
for t in range(5, 26):
    L.run(1)   # timestep t + 1; the block times are the last launch's
    torch.cuda.synchronize()
    if t + 1 not in (6, 15, 25):
        continue
    nb = 2048
    buf = np.zeros(2 * nb, dtype=np.uint64)
    assert f(buf.ctypes.data, 2 * nb) == 0
    st, en = buf[0::2].astype(np.int64), buf[1::2].astype(np.int64)
    t0 = st.min()
    st, en = (st - t0) * 10e-3, (en - t0) * 10e-3   # us (100 MHz)
    dur = en - st
    span = en.max()
    order = np.argsort(st)
    print(f"timestep {t + 1}: launch span {span:.2f} us (first start to last end), block life mean {dur.mean():.2f} "
          f"median {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f} us; "
          f"sum of block lives / 768 slots = {dur.sum() / 768:.2f} us")
    grid = np.arange(0, span + 1, 1.0)
    act = [(int(((st <= x) & (en > x)).sum())) for x in grid]
    print("  resident blocks per us:", " ".join(str(a) for a in act))
    last = np.argsort(en)[-10:]
    print("  last 10 blocks to end (blockIdx, start, end):",
          " ".join(f"({b},{st[b]:.1f},{en[b]:.1f})" for b in last))
    slow = np.argsort(dur)[-8:]
    print("  8 longest-lived (blockIdx, life):", " ".join(f"({b},{dur[b]:.1f})" for b in slow))
