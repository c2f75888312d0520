"""A/B timing of the fused lattice step for two source trees (tools/_ab/<tree>): the same
jittered lattice, hipGraph replay, step time and advance-phase time by HIP events.
Usage: python tools/ab_lattice.py <tree-root> <spacing> [steps] [rows] [rw]  (1024 x rows agents;
rw: cfg4r's random-walk nominal control, amplitude 1, seed 5)"""
import sys
import time

root, spacing = sys.argv[1], float(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
sys.path.insert(0, root)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

W = 1024
H = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
rng = np.random.default_rng(0)
r, c = np.divmod(np.arange(W * H), W)
pos = np.stack([c * spacing, r * spacing], axis=1).astype(np.float64)
pos += rng.uniform(-spacing / 2, spacing / 2, size=pos.shape)
rw = len(sys.argv) > 5 and sys.argv[5] == "rw"
L = swarm.LatticeSwarm(pos, W, H, gain=0.25, nominal=("random", 1.0, 5) if rw else None)
L.capture()
for _ in range(20):
    L.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    L.step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
ks = []
for _ in range(10):
    L.build_phase()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    L.advance_phase()
    b.record()
    ks.append((a, b))
torch.cuda.synchronize()
adv = np.mean([a.elapsed_time(b) for a, b in ks]) * 1e3
run = ""
if hasattr(L, "run"):  # trees with cbf_lattice_run: graphs of 10-timestep calls
    L.capture(steps=10)
    for _ in range(2):
        L.run(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // 10):
        L.run(10)
    torch.cuda.synchronize()
    run = f", run(10) {(time.perf_counter() - t0) / (steps // 10 * 10) * 1e6:.1f} us/step"
print(f"{root} spacing {spacing} rows {H}{' rw' if rw else ''}: step {dt * 1e6:.1f} us, advance {adv:.1f} us{run}")
