"""torch.ops.cbf_amd.* (the thin PyTorch-ROCm extension over the C ABI) on the GPU: the same results
as the golden vectors and the oracle, bit-identical to the ctypes path, on the current stream, and
capturable in a hipGraph."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from cbf_amd import scenarios, swarm, torch_ops  # noqa: E402
from oracle import coracle, pyoracle as po  # noqa: E402

DEV = torch.device("cuda")
OPS = torch_ops.ops()


def _t(a, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=DEV)


def test_get_safe_control_batch_op_vs_golden(golden):
    F = golden("golden_filter.npz")
    for ms, dmin, k in {(float(a), float(b), float(c)) for a, b, c in zip(F["max_speed"], F["dmin"], F["k"])}:
        idx = [i for i in range(len(F["r"])) if (F["max_speed"][i], F["dmin"][i], F["k"][i]) == (ms, dmin, k)
               and np.array_equal(F["g"][i], 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]]))
               and not F["f"][i].any()]   # the op takes the callers' f and g (torch_ops.cpp)
        if not idx:
            continue
        obs = [F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]] for i in idx]
        off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int32)
        u, st = OPS.get_safe_control_batch(_t(F["r"][idx]), _t(F["u0"][idx]), _t(off, torch.int32),
                                           _t(np.vstack(obs) if len(np.vstack(obs)) else np.zeros((0, 4))),
                                           ms, dmin, k)
        u = u.cpu().numpy()
        for t, i in enumerate(idx):
            assert np.abs(u[t] - F["u"][i]).max() <= 1e-12, i
            ref = coracle.filter_one(po.Params(ms, dmin, k), F["r"][i], obs[t], F["u0"][i])
            assert np.array_equal(u[t], ref["u"]), i


def test_filter_swarm_op_vs_oracle():
    rng = np.random.default_rng(3)
    pos = rng.uniform(-1.5, 1.5, (700, 2))
    vel = rng.normal(0, 0.3, (700, 2))
    u, st, cnt = OPS.filter_swarm(_t(pos), _t(vel), 100, 15.0)
    ref = coracle.filter_swarm(po.Params(15), pos, vel, 100)
    assert np.array_equal(u.cpu().numpy(), ref["u"])
    assert np.array_equal(st.cpu().numpy(), ref["status"])
    assert np.array_equal(cnt.cpu().numpy(), ref["cnt"])


def test_lattice_step_op_matches_ctypes_path_and_graph_captures():
    W, H = 96, 80
    pos = scenarios.lattice(W, H, seed=4)
    L = swarm.LatticeSwarm(pos, W, H)
    g = L.grid
    args = (W, H, L.gain, L.T, g.x0, g.y0, 1 / g.inv_h, g.nx, g.ny)
    ws = torch.zeros(OPS.lattice_workspace_size(W, H, g.x0, g.y0, 1 / g.inv_h, g.nx, g.ny), dtype=torch.uint8,
                     device=DEV)
    stats = torch.zeros(1024, dtype=torch.int64, device=DEV)
    P = _t(pos)
    for _ in range(3):
        L.step()
        vel, u, st, cnt = OPS.lattice_step(P, *args, ws, stats)
    torch.cuda.synchronize()
    assert torch.equal(P, L.pos) and torch.equal(u, L.u) and torch.equal(st, L.status)
    # step 4 on a side stream (warm-up), then captured into a hipGraph (the capture runs nothing)
    # and replayed 4 times: 8 steps in all, the same trajectory as 8 ctypes steps
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        OPS.lattice_step(P, *args, ws, stats)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = OPS.lattice_step(P, *args, ws, stats)
    for _ in range(4):
        graph.replay()
    torch.cuda.synchronize()
    ref = swarm.LatticeSwarm(pos, W, H)
    for _ in range(8):
        ref.step()
    torch.cuda.synchronize()
    assert torch.equal(P, ref.pos) and torch.equal(out[1], ref.u) and torch.equal(out[2], ref.status)


def test_lattice_run_op_equals_step_ops():
    """torch.ops.cbf_amd.lattice_run(k), with either cull, == k lattice_step ops, bit for bit
    (positions, the last timestep's outputs, the decoded statistics)."""
    from cbf_amd import _lib
    W, H = 128, 96
    pos = scenarios.lattice(W, H, seed=6, spacing=0.2)
    L = swarm.LatticeSwarm(pos, W, H)
    g = L.grid
    geo = (g.x0, g.y0, 1 / g.inv_h, g.nx, g.ny)
    nb = OPS.lattice_workspace_size(W, H, *geo)
    outs = []
    for run in ("steps", "run", "run_window"):
        ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
        stats = torch.zeros(1024, dtype=torch.int64, device=DEV)
        P = _t(pos)
        if run == "steps":
            for _ in range(7):
                out = OPS.lattice_step(P, W, H, L.gain, L.T, *geo, ws, stats)
        else:   # (window_cull: the lattice-window cull, CBF_RUN_WINDOW_CULL)
            out = OPS.lattice_run(P, W, H, L.gain, L.T, 7, *geo, ws, stats, window_cull=run == "run_window")
        torch.cuda.synchronize()
        outs.append((P, out, _lib.decode_stats(stats.cpu().numpy())))
    pa, oa, sa = outs[0]
    for pb, ob, sb in outs[1:]:
        assert torch.equal(pa, pb) and all(torch.equal(x, y) for x, y in zip(oa, ob)) and sa == sb
    assert sa["solves"] > 0 and sa["errors"] == 0


def test_lattice_ops_without_stats_and_argument_checks():
    """stats=None reaches the statistics-free kernels (the bench's timed instantiation): the same
    positions and outputs as with statistics; steps=0 and tensors on another device are rejected."""
    W, H = 96, 64
    pos = scenarios.lattice(W, H, seed=9)
    L = swarm.LatticeSwarm(pos, W, H)
    g = L.grid
    geo = (g.x0, g.y0, 1 / g.inv_h, g.nx, g.ny)
    nb = OPS.lattice_workspace_size(W, H, *geo)
    outs = []
    for stats in (torch.zeros(1024, dtype=torch.int64, device=DEV), None):
        ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
        P = _t(pos)
        out = OPS.lattice_run(P, W, H, L.gain, L.T, 5, *geo, ws, stats)
        out2 = OPS.lattice_step(P, W, H, L.gain, L.T, *geo, ws, stats)
        torch.cuda.synchronize()
        outs.append((P, out, out2))
    (pa, oa, qa), (pb, ob, qb) = outs
    assert torch.equal(pa, pb)
    assert all(torch.equal(x, y) for x, y in zip(oa + qa, ob + qb))
    ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
    with pytest.raises(RuntimeError, match="steps"):
        OPS.lattice_run(_t(pos), W, H, L.gain, L.T, 0, *geo, ws, None)
    with pytest.raises(RuntimeError, match="workspace"):
        OPS.lattice_step(_t(pos), W, H, L.gain, L.T, *geo, torch.zeros(nb, dtype=torch.uint8), None)
