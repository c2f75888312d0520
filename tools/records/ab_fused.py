"""A/B timing of a window-cull run's queued-QP placement, in one process (the switch is a runtime
field, cbf_params.launch_flags CBF_LAUNCH_QUEUE_KERNEL): hipGraphs of run(20) with the queued QPs
solved by the next timestep's build ("next_build") or by the queue kernel after every filter
("queue_kernel"), statistics off as the bench times them, interleaved repetitions; the end states
must agree.  Usage: python tools/ab_fused.py [spacing ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

W = H = 1024
for sp in [float(a) for a in sys.argv[1:]] or [0.145, 0.2]:
    pos = scenarios.lattice(W, H, seed=0, spacing=sp)
    runs = {}
    for hs in ("next_build", "queue_kernel"):
        L = swarm.LatticeSwarm(pos, W, H, gain=scenarios.LATTICE_GAIN, cull="window",
                               params=swarm.FilterParams(hard_solve=hs))
        L.collect_stats = False
        L.run(5)
        L.capture(steps=20)
        runs[hs] = L
    torch.cuda.synchronize()
    times = {hs: [] for hs in runs}
    for rep in range(6):
        for hs, L in (runs.items() if rep % 2 == 0 else reversed(list(runs.items()))):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L.run(20)
            torch.cuda.synchronize()
            times[hs].append((time.perf_counter() - t0) / 20 * 1e6)
    a, b = (runs[k].pos.cpu().numpy() for k in ("next_build", "queue_kernel"))
    same = bool(np.array_equal(a, b))
    print(f"spacing {sp}: run(20) us/step " + ", ".join(f"{k} {min(v):.1f} (median {np.median(v):.1f})"
                                                       for k, v in times.items()) + f"; end states equal: {same}",
          flush=True)
