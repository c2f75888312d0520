"""Rollout checkpoints (save the SoA state .npz every K steps): a lattice swarm saved
mid-rollout and rebuilt from the file continues the rollout bit for bit -- positions, controls,
statuses, neighbour counts and the statistics totals -- for the consensus and the random-walk
nominal controls, through step() and run()."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU boxes but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from cbf_amd import _lib, scenarios, swarm  # noqa: E402


@pytest.mark.parametrize("nominal,spacing,cull", [(None, 0.145, "cells"), (("random", 1.0, 5), 0.22, "cells"),
                                                 (None, 0.145, "window")])
def test_lattice_checkpoint_resumes_bit_identical(tmp_path, nominal, spacing, cull):
    W, H = 96, 64
    A = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=3, spacing=spacing), W, H, nominal=nominal, cull=cull)
    A.run(7)
    A.step()
    path = str(tmp_path / "ck.npz")
    A.save_checkpoint(path)
    B = swarm.LatticeSwarm.from_checkpoint(path)
    for S in (A, B):
        S.run(9)
        S.step()
    torch.cuda.synchronize()
    for a, b in ((A.pos, B.pos), (A.u, B.u), (A.status, B.status), (A.nbr_count, B.nbr_count),
                 (A.vel, B.vel)):
        assert torch.equal(a, b)
    # the statistics words are spread over slots by the order of the queue's atomics; their totals
    # and extrema (what decode_stats reads) are deterministic
    assert _lib.decode_stats(A.stats.cpu().numpy()) == _lib.decode_stats(B.stats.cpu().numpy())
    assert B.grid.nx == A.grid.nx and B.grid.inv_h == A.grid.inv_h and B.nominal == A.nominal
    assert B.cull == A.cull


def _tamper(tmp_path, path, name, fn):
    with np.load(path, allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    fn(arrays)
    bad = str(tmp_path / f"bad_{name}.npz")
    np.savez(bad, **arrays)
    return bad


def test_checkpoint_refuses_another_shape(tmp_path):
    """from_checkpoint's own checks (not the constructor's): a truncated workspace array, a state
    array of another dtype, and metadata from another workspace layout or ABI are refused with the
    checkpoint's error."""
    import json
    A = swarm.LatticeSwarm(scenarios.lattice(32, 32, seed=1), 32, 32)
    A.step()
    path = str(tmp_path / "ck.npz")
    A.save_checkpoint(path)
    B = swarm.LatticeSwarm.from_checkpoint(path)     # the untouched file loads
    assert torch.equal(A.ws, B.ws)

    def meta(**kw):
        def f(arrays):
            m = json.loads(bytes(arrays["meta"]).decode())
            m.update(kw)
            arrays["meta"] = np.frombuffer(json.dumps(m).encode(), dtype=np.uint8)
        return f

    def trunc(arrays):
        arrays["state5"] = arrays["state5"][:-256]      # the workspace

    def dtype(arrays):
        arrays["state6"] = arrays["state6"].astype(np.float64)   # the statistics words
    for name, fn, msg in (("ws", trunc, "state5"), ("dtype", dtype, "state6"),
                          ("layout", meta(workspace_layout=-1), "workspace_layout"),
                          ("abi", meta(abi_version=-1), "abi_version"),
                          ("bytes", meta(ws_bytes=1), "workspace of 1 bytes")):
        with pytest.raises(ValueError, match=msg):
            swarm.LatticeSwarm.from_checkpoint(_tamper(tmp_path, path, name, fn))
