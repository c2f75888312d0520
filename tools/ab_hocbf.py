"""A/B driver (GPU): 40 HOCBF-mode timesteps of the cfg4 lattice from the source tree given
(argv[1]), graph-replayed in one 20-step graph after a 20-step warm-up; prints the end state's
sha256 prefix.  Kernel times come from the rocprofv3 trace around it (tools/gpu_ab_hocbf_trace.sh)."""
import hashlib
import sys

tree = sys.argv[1] if len(sys.argv) > 1 else "."
sys.path.insert(0, tree)
import torch  # noqa: E402
from cbf_amd import scenarios, swarm  # noqa: E402

W = H = 1024
S = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0), W, H, gain=scenarios.LATTICE_GAIN, barrier="euclidean_hocbf")
S.collect_stats = False
S.run(20)
S.capture(steps=20)
S.run(20)
torch.cuda.synchronize()
print("end", hashlib.sha256(S.pos.cpu().numpy().tobytes()).hexdigest()[:12], swarm.__file__)
