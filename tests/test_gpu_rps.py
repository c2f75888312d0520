"""rps-lite on the HIP path against the restatement in oracle/rps_lite.py:
the exact coupled certificate QP (Goldfarb-Idnani, one wavefront per scenario), the unicycle
maps / step, and cross_and_rescue.py's whole loop as shipped.  Floating-point tolerances are
stated per test: the certificate's pivots and rotations run in a different order than numpy's,
and the GPU's sin / cos / atan2 are not glibc's, so agreement is to rounding, not bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from cbf_amd import rps  # noqa: E402
from oracle import pyoracle as po, rps_lite as R  # noqa: E402

from .test_rps_oracle import cert_cases  # noqa: E402

DEV = torch.device("cuda")
X_TOL = 1e-9      # certificate solution: |x_gpu - x_oracle| <= X_TOL * max(1, |x|)


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=DEV)


def test_cert_batch_vs_oracle():
    rng = np.random.default_rng(11)
    cert = rps.SiBarrierCert(safety_radius=0.12)
    by_n = {}
    for dxi, x in cert_cases(rng, 400):
        by_n.setdefault(dxi.shape[1], []).append((dxi, x))
    checked = 0
    for N, cases in sorted(by_n.items()):
        D = np.stack([c[0].T for c in cases])
        X = np.stack([c[1].T for c in cases])
        res = cert.batch(_t(D), _t(X), iters=True)
        out, st = res["out"].cpu().numpy(), res["status"].cpu().numpy()
        for t, (dxi, x) in enumerate(cases):
            ref, info = R.si_barrier_cert(dxi, x, safety_radius=0.12)
            assert st[t] == info["status"], (N, t)
            err = np.abs(out[t].T - ref).max()
            assert err <= X_TOL * max(1.0, np.abs(ref).max()), (N, t, err)
            if st[t] == R.CERT_OPTIMAL:
                # the GPU answer itself satisfies the QP's rows (independent of the oracle)
                v = out[t].reshape(-1)
                assert np.max(info["A"] @ v - info["b"]) <= 1e-9 * max(1.0, np.abs(info["b"]).max())
            checked += 1
    assert checked == 400


def test_cert_call_surface_matches_rps_shape():
    f = rps.create_single_integrator_barrier_certificate_with_boundary(safety_radius=0.12)
    x = np.array([[-0.3, -0.2, 0.4, 0.5], [0.0, 0.05, 0.1, -0.4]])
    dxi = np.array([[0.2, -0.2, 0.0, 0.05], [0.0, 0.0, -0.1, 0.1]])
    out = f(dxi, x)
    ref, _ = R.si_barrier_cert(dxi, x, safety_radius=0.12)
    assert out.shape == (2, 4) and np.abs(out - ref).max() <= 1e-12


def test_cert_infeasible_and_argument_errors():
    cert = rps.SiBarrierCert(safety_radius=0.12)
    # boundary rows alone infeasible: an agent far outside the arena on both sides is impossible,
    # so use a degenerate arena whose +x and -x rows contradict
    bad = rps.SiBarrierCert(safety_radius=0.12, boundary_points=(1.0, -1.0, -1.0, 1.0))
    d = _t(np.array([[[0.1, 0.0]]]))
    x = _t(np.array([[[0.0, 0.0]]]))
    r = bad.batch(d, x)
    ref = R.goldfarb_idnani(*R.si_barrier_qp(np.array([[0.1], [0.0]]), np.array([[0.0], [0.0]]), safety_radius=0.12,
                                             boundary_points=(1.0, -1.0, -1.0, 1.0)))
    assert int(r["status"][0]) == ref["status"] == R.CERT_INFEASIBLE
    assert np.array_equal(r["out"][0].cpu().numpy(), [[0.1, 0.0]])
    with pytest.raises(Exception):
        cert.batch(_t(np.zeros((1, 33, 2))), _t(np.zeros((1, 33, 2))))


def test_unicycle_kernels_vs_oracle():
    rng = np.random.default_rng(12)
    n = 4096
    poses = np.vstack([rng.uniform(-1.5, 1.5, (2, n)), rng.uniform(-np.pi, np.pi, n)])
    dxi = rng.normal(0, 0.5, (2, n))
    si_to_uni, uni_to_si = rps.create_si_to_uni_mapping()
    assert np.abs(uni_to_si(poses) - R.uni_to_si_states(poses)).max() <= 1e-15
    dxu_ref = R.si_to_uni_dyn(dxi, poses)
    assert np.abs(si_to_uni(dxi, poses) - dxu_ref).max() <= 1e-12
    u = rps.unicycle_params()
    p = _t(poses.T)
    rps.unicycle_advance(u, p, _t(dxi.T), mode=0)
    ref = R.unicycle_step(poses, R.set_velocities(dxu_ref))
    got = p.cpu().numpy().T
    dth = np.abs(np.angle(np.exp(1j * (got[2] - ref[2]))))
    assert np.abs(got[:2] - ref[:2]).max() <= 1e-14 and dth.max() <= 1e-12
    # Robotarium protocol: set_velocities (v, w) then step
    rb = rps.Robotarium(n, poses)
    rb.set_velocities(np.arange(n), dxu_ref)
    rb.step()
    got2 = rb.get_poses()
    assert np.abs(got2[:2] - ref[:2]).max() <= 1e-14


def test_cross_and_rescue_shipped_teacher_forced():
    """Each GPU step starts from the oracle's state of that step (teacher forcing), so rounding
    differences cannot compound: per-step outputs agree to rounding for 300 steps."""
    p = po.Params(15)
    sim = rps.CrossAndRescue()
    poses, obs = R.cross_and_rescue_initial()
    worst = 0.0
    for k in range(300):
        sim.poses.copy_(_t(poses.T))
        sim.obs_pos.copy_(_t(obs.T))
        g = sim.step()
        poses_n, obs_n, rec = R.cross_and_rescue_step(poses, obs, p)
        assert np.array_equal(g["nbr_count"].cpu().numpy(), rec["cnt"]), k
        assert np.array_equal(g["status"].cpu().numpy() & 0xFF, rec["status"] & 0xFF), k
        e = max(np.abs(g["nominal"].cpu().numpy().T - rec["nominal"]).max(),
                np.abs(g["filtered"].cpu().numpy().T - rec["filtered"]).max(),
                np.abs(g["cert"].cpu().numpy().T - rec["cert"]).max(),
                np.abs(sim.poses.cpu().numpy().T[:2] - poses_n[:2]).max(),
                np.abs(sim.obs_pos.cpu().numpy().T - obs_n).max())
        worst = max(worst, e)
        assert e <= 1e-9, (k, e)
        poses, obs = poses_n, obs_n
    assert worst <= 1e-9


def test_cross_and_rescue_shipped_free_run():
    """Free-running GPU rollout vs the oracle's: stays within 1e-6 over 200 steps and keeps the
    robots inside the arena (the certificate's boundary rows)."""
    p = po.Params(15)
    sim = rps.CrossAndRescue()
    poses, obs = R.cross_and_rescue_initial()
    for k in range(200):
        sim.step()
        poses, obs, _ = R.cross_and_rescue_step(poses, obs, p)
    got = sim.poses.cpu().numpy().T
    assert np.abs(got[:2] - poses[:2]).max() <= 1e-6
    assert np.all(np.abs(got[0]) <= 1.6) and np.all(np.abs(got[1]) <= 1.0)


def test_meet_at_center_shipped_teacher_forced():
    """meet_at_center.py as shipped (10 unicycle robots, no certificate), per-step outputs from the
    oracle's state of that step: filter decisions identical, values to rounding, 300 steps."""
    p = po.Params(15)
    sim = rps.MeetAtCenter()
    poses = R.meet_at_center_initial(10)
    filtered = 0
    for k in range(300):
        sim.poses.copy_(_t(poses.T))
        g = sim.step()
        poses_n, rec = R.meet_at_center_step(poses, p)
        assert np.array_equal(g["nbr_count"].cpu().numpy(), rec["cnt"]), k
        assert np.array_equal(g["status"].cpu().numpy() & 0xFF, rec["status"] & 0xFF), k
        e = max(np.abs(g["nominal"].cpu().numpy().T - rec["nominal"]).max(),
                np.abs(g["filtered"].cpu().numpy().T - rec["filtered"]).max(),
                np.abs(sim.poses.cpu().numpy().T[:2] - poses_n[:2]).max())
        assert e <= 1e-9, (k, e)
        filtered += int((rec["cnt"] > 0).sum())
        poses = poses_n
    assert filtered > 0          # the filter did run during the rollout
