"""Per-call time of the drop-in ControlBarrierFunction.get_safe_control (the reference's
one-ego-at-a-time call surface, cbf.py:18-92) on the GPU: a cfg2-like ego with 6 obstacles.
Usage: python tools/compat_call_time.py [tree-root] [calls]"""
import sys
import time

root = sys.argv[1] if len(sys.argv) > 1 else "."
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
sys.path.insert(0, root)
import numpy as np  # noqa: E402
import cbf_amd  # noqa: E402

rng = np.random.default_rng(0)
c = cbf_amd.ControlBarrierFunction(15)
f, g = np.zeros((4, 4)), 0.1 * np.array([[1.0, 0], [0, 1], [0, 0], [0, 0]])
r = rng.uniform(-1, 1, 4)
obs = r + rng.uniform(-0.2, 0.2, (6, 4))
u0 = rng.uniform(-1, 1, 2)
for _ in range(50):
    c.get_safe_control(r, obs, f, g, u0)
t0 = time.perf_counter()
for _ in range(calls):
    u = c.get_safe_control(r, obs, f, g, u0)
dt = (time.perf_counter() - t0) / calls
print(f"{root}: get_safe_control {dt * 1e6:.1f} us per call, u = {u}")
