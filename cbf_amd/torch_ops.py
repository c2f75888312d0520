"""torch.ops.cbf_amd.*: the thin PyTorch-ROCm extension over the C ABI (csrc/torch_ops.cpp,
built in-tree as libcbf_amd_torch.so).  The ops run on the current HIP stream, allocate their
outputs with torch's caching allocator and can be captured in a hipGraph (torch.cuda.graph):

  get_safe_control_batch(robot_state, u0, nbr_off, obs_states, max_speed, dmin=0.2, k=1, f=None, g=None)
      -> (u, status)                                   ControlBarrierFunction.get_safe_control, cbf.py:18-92
  filter_swarm(pos, vel, n_obs, max_speed, dmin=0.2, k=1, safety_distance=0.2)
      -> (u, status, nbr_count)                        cross_and_rescue.py:135-160 (all-pairs cull)
  lattice_step(pos, W, H, gain, T, x0, y0, cell, nx, ny, workspace, stats, max_speed=15, ...)
      -> (nominal, u, status, nbr_count)               one fused timestep, pos advanced in place
  lattice_workspace_size(W, H, x0, y0, cell, nx, ny) -> int
  abi_version() -> int

Like the ctypes binding there is no CPU fallback: the ops exist only for GPU tensors.
"""
from __future__ import annotations

import os

import torch

from . import _lib  # noqa: F401  (loads libcbf_amd.so first; the extension links against it)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcbf_amd_torch.so")
_loaded = False


def ops():
    """The torch.ops.cbf_amd namespace (loads the extension once; raises if it is not built)."""
    global _loaded
    if not _loaded:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              "g.build()'`")
        torch.ops.load_library(LIB_PATH)
        _loaded = True
    return torch.ops.cbf_amd
