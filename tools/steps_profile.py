"""Per-timestep kernel durations over the first timesteps of the cfg4 rollout (run under
rocprofv3 --kernel-trace; tools/gpu_steps_profile.sh analyses the trace)."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

W = H = 1024
S = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H)
S.collect_stats = False
S.run(40)
torch.cuda.synchronize()
