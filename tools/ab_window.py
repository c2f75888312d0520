"""A/B timing of the lattice step for a source tree (tools/_ab/<tree> or .): hipGraphs of run(10),
per-timestep time, and the build / filter / advance kernels by HIP events (the filter's end event
recorded by the advance call).  Usage: python tools/ab_window.py <tree-root> <cull> [spacing] [rows] [placement]"""
import os
import sys
import time

root, cull = sys.argv[1], sys.argv[2]
spacing = float(sys.argv[3]) if len(sys.argv) > 3 else 0.145
H = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
placement = sys.argv[5] if len(sys.argv) > 5 else "auto"
sys.path.insert(0, root)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

W = 1024
L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0, spacing=spacing), W, H, gain=0.25, cull=cull,
                       params=swarm.FilterParams(solve_placement=placement,
                                                 window_guard=os.environ.get("AB_GUARD", "auto")))
L.collect_stats = False
if os.environ.get("AB_DRIVER"):
    # the driver's timed span: timesteps 6-25 (bench.py --steps 20 --warmup 5), as two run(10) graph
    # replays from the state after 5 timesteps, repeated from a snapshot
    L.run(5)
    snap = L.snapshot()
    L.capture(steps=10)
    reps, t = 5, 0.0
    for _ in range(reps):
        L.restore(snap)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.run(10)
        L.run(10)
        torch.cuda.synchronize()
        t += time.perf_counter() - t0
    run = t / (20 * reps) * 1e6
else:
    L.capture(steps=10)
    for _ in range(3):
        L.run(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        L.run(10)
    torch.cuda.synchronize()
    run = (time.perf_counter() - t0) / 100 * 1e6
ev = []
for _ in range(10):
    a, m, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    m.record()
    torch.cuda._sleep(200000)   # the GPU busy while the host enqueues: events time kernels, not launches
    a.record()
    L.build_phase()
    torch.cuda._sleep(200000)
    b.record()
    L.advance_phase(mark=m, commit=False) if cull == "window" else L.advance_phase(mark=m)
    c.record()
    ev.append((a, m, b, c))
torch.cuda.synchronize()
bld = np.mean([a.elapsed_time(b) for a, m, b, c in ev]) * 1e3
flt = np.mean([b.elapsed_time(m) for a, m, b, c in ev]) * 1e3
adv = np.mean([b.elapsed_time(c) for a, m, b, c in ev]) * 1e3
print(f"{root} {cull} {placement} spacing {spacing} rows {H}: run(10) {run:.1f} us/step, build {bld:.1f}, filter {flt:.1f}, "
      f"advance {adv:.1f} us", flush=True)
