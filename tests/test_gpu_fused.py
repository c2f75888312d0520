"""The queued QPs of a window-cull run solved by the next timestep's build (cbf_amd/csrc/window.hip
k_window_prep FU, FusedHard; include/cbf_amd.h CBF_LAUNCH_QUEUE_KERNEL for the other form) instead
of by the queue kernel after every filter.  The solve is the reference's QP (cbf.py:75-87) with its
+1 rule, the rolled plane loop (solve_planes_rolled) instead of the unrolled one: every timestep's
outputs must equal the queue kernel's and the oracle's bit for bit, including history outputs
(the reference's per-step si_velocities), odd / even step counts, graph replay, the random-walk
regime where a build's three rows hold more queued QPs than it has threads (chunks), and the
parameter sets of tests/paramsets.py (f != 0 kernels)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU boxes but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from cbf_amd import scenarios, swarm  # noqa: E402
from oracle import coracle  # noqa: E402
from tests import paramsets  # noqa: E402

GAIN = 0.25


def _pair(pos, W, H, pset="callers", nominal=None, placement="queued"):
    """Two window-cull swarms, statistics off (the fused form's condition): next-build vs queue kernel."""
    out = []
    for hs in ("next_build", "queue_kernel"):
        L = swarm.LatticeSwarm(pos, W, H, gain=GAIN, nominal=nominal, cull="window",
                               params=paramsets.filter_params(pset, solve_placement=placement, hard_solve=hs))
        L.collect_stats = False
        out.append(L)
    return out


def _same(A, B, hist=None):
    """The end state and the outputs; after a history run the outputs are the history arrays (the
    swarms' own output tensors are not written by it)."""
    pairs = ((A.pos, B.pos),) if hist else \
        ((A.pos, B.pos), (A.vel, B.vel), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count))
    for x, y in pairs:
        assert torch.equal(x, y)
    if hist:
        for x, y in zip(A.history(hist), B.history(hist)):
            assert torch.equal(x, y)


@pytest.mark.parametrize("pset", paramsets.NAMES)
@pytest.mark.parametrize("steps", [2, 3, 6])
def test_fused_run_equals_queue_kernel_and_oracle(pset, steps):
    """run(steps, history=True): every timestep's nominal control, u, status and neighbour count and
    the final positions == the queue-kernel form's == the oracle's rollout."""
    W, H = 160, 96
    pos = scenarios.lattice(W, H, seed=31, spacing=0.16)
    A, B = _pair(pos, W, H, pset)
    for L in (A, B):
        L.run(steps, history=True)
    torch.cuda.synchronize()
    _same(A, B, steps)
    vel_h, u_h, st_h, cnt_h = (t.cpu().numpy() for t in A.history(steps))
    ref = pos.copy()
    p = paramsets.oracle_params(pset)
    solved = 0
    for t in range(steps):
        vel = coracle.consensus_lattice(W, H, 0, H, ref, GAIN)
        o = coracle.filter_swarm(p, ref, vel, 0)
        assert np.array_equal(vel_h[t], vel), t
        assert np.array_equal(u_h[t], o["u"]), t
        assert np.array_equal(st_h[t], o["status"]), t
        assert np.array_equal(cnt_h[t], o["cnt"]), t
        solved += int(((o["status"] & 0xFF) != 0).sum())
        ref = coracle.euler(ref, o["u"], 1 / 30)
    assert np.array_equal(A.pos.cpu().numpy(), ref)
    assert solved > 0


@pytest.mark.parametrize("W,H,steps", [(1024, 264, 4), (1000, 20, 3), (64, 16, 5)])
def test_fused_random_walk_many_queued(W, H, steps):
    """cfg4r's random walk at spacing 0.22: about 10 % of the QPs go to the queue, so a build block
    solves more queued QPs of its three rows than it has threads (the chunked path) at W = 1024;
    a width that is not a multiple of the 64-column tile; both step parities; the last timestep
    (queue kernel) and the inner ones (next build) against the queue-kernel form every timestep."""
    pos = scenarios.lattice(W, H, seed=32, spacing=0.22)
    A, B = _pair(pos, W, H, nominal=("random", 1.0, 9))
    for L in (A, B):
        L.run(steps, history=True)
        L.run(1)
    torch.cuda.synchronize()
    _same(A, B)
    _same(A, B, steps)
    st = A.history(steps)[2].cpu().numpy()
    assert ((st & 0xFF) != 0).sum() > 0


def test_fused_graph_replay_and_odd_even():
    """Graph capture of run(5) and of run(4) (the ping-pong's two parities), replayed, == the queue
    kernel form's, and the fused form launches no queue kernel for the inner timesteps (its
    result equals a run of single steps too)."""
    W, H = 256, 128
    pos = scenarios.lattice(W, H, seed=33, spacing=0.145)
    A, B = _pair(pos, W, H)
    C = swarm.LatticeSwarm(pos, W, H, gain=GAIN, cull="window", params=swarm.FilterParams(solve_placement="queued"))
    C.collect_stats = False
    for L in (A, B):
        L.capture(steps=5)
        L.run(5)
        L.capture(steps=4)
        L.run(4)
    for _ in range(5 + 5 + 4 + 4):
        C.step()
    torch.cuda.synchronize()
    _same(A, B)
    for x, y in ((A.pos, C.pos), (A.u, C.u), (A.status, C.status)):
        assert torch.equal(x, y)


def test_fused_full_size_cfg4_driver_span():
    """cfg4 at full size (1024 x 1024), 25 timesteps as bench.py runs them (statistics off, 5 + 20
    in graphs of 20): the fused form's end state == the queue-kernel form's bit for bit."""
    W = H = 1024
    pos = scenarios.lattice(W, H, seed=0)
    res = []
    for hs in ("next_build", "queue_kernel"):
        L = swarm.LatticeSwarm(pos, W, H, cull="window", params=swarm.FilterParams(hard_solve=hs))
        L.collect_stats = False
        L.run(5)
        L.run(20)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (L.pos, L.vel, L.u, L.status, L.nbr_count)])
        del L
    for a, b in zip(*res):
        assert np.array_equal(a, b)
