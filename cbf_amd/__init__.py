"""cbf_amd -- MI355X-native CBF safety filter (hand-written HIP for gfx950 behind a C ABI).

Drop-in for the reference's hot path (YilunAllenChen/CBF): ``ControlBarrierFunction``
(cbf.py:5-92) plus batched swarm steps for the callers' per-agent loop
(cross_and_rescue.py:97-175, meet_at_center.py:76-153).  See DESIGN.md.
"""
from ._lib import (STATUS_BOX_INFEASIBLE, STATUS_IDLE, STATUS_NBR_OVERFLOW, STATUS_OPTIMAL, STATUS_RELAX_CAP,  # noqa
                   STATUS_RELAXED,  # noqa
                   CbfError, lib)
from .cbf import ControlBarrierFunction  # noqa: F401
from .swarm import (FilterParams, GroupSwarm, LatticeSwarm, consensus_csr, consensus_lattice, euler,  # noqa
                    filter_swarm, filter_swarm_hocbf, grid_for_points, make_grid, mc_rollout)
