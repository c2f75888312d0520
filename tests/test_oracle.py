"""The oracle (CPU restatement) against the golden vectors captured from the
reference's own cbf.py (tests/golden/make_golden.py), and C oracle == Python
oracle bit-for-bit.  CPU only."""
import numpy as np
import pytest

from oracle import coracle, pyoracle as po
from tests.golden import qp_bruteforce


def _cases(F):
    for i in range(len(F["r"])):
        p = po.Params(F["max_speed"][i], F["dmin"][i], F["k"][i], g=F["g"][i], f=F["f"][i])
        obs = F["obs"][F["obs_off"][i]:F["obs_off"][i + 1]]
        A0 = F["A"][F["ab_off"][i]:F["ab_off"][i + 1]]
        b0 = F["b"][F["ab_off"][i]:F["ab_off"][i + 1]]
        yield i, p, obs, A0, b0


@pytest.mark.parametrize("impl", ["py", "c"])
def test_assembly_bit_exact_vs_reference(golden, impl):
    """A and b handed to cvxopt (cbf.py:72-81) reproduced bit-for-bit."""
    F = golden("golden_filter.npz")
    asm = po.assemble if impl == "py" else coracle.assemble
    n = 0
    for i, p, obs, A0, b0 in _cases(F):
        A, b = asm(p, F["r"][i], obs, F["u0"][i])
        assert np.array_equal(A, A0), i
        assert np.array_equal(b, b0), i
        n += 1
    assert n == len(F["r"]) > 2900


def test_golden_covers_the_reference_parameters(golden):
    """The fixtures exercise every input of ControlBarrierFunction (cbf.py:6) and of
    get_safe_control's rows (cbf.py:55-59) away from the callers' defaults: random f (L_f),
    random g, non-integer k, other dmin / max_speed -- and both at once."""
    F = golden("golden_filter.npz")
    fz = np.abs(F["f"]).reshape(len(F["r"]), -1).max(axis=1) == 0
    kint = F["k"] == np.round(F["k"])
    gdef = np.all(F["g"] == 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]]), axis=(1, 2))
    assert (~fz).sum() >= 500 and (~kint).sum() >= 400 and (~gdef).sum() >= 450
    both = ~fz & ~kint & ~gdef & (F["dmin"] != 0.2)
    assert both.sum() >= 100
    # and the non-default cases include infeasible (relaxed) QPs and binding minimisers
    assert (F["relax_iters"][~fz] > 0).sum() > 50 and (np.abs(F["x"][~fz]).max(axis=1) > 0).sum() > 50


@pytest.mark.parametrize("impl", ["py", "c"])
def test_filter_vs_reference(golden, impl):
    """x within 1e-12 of the KKT-certified minimiser; u = reference de-bias+clip (cbf.py:89-91)
    within 1e-12.  Infeasible QPs (cvxopt's output undefined, cbf.py:82 never reads the status)
    must be detected and resolved by the reference's own +1 retry rule (cbf.py:84-87) with the
    same relaxation count as the independent brute-force restatement."""
    F = golden("golden_filter.npz")
    flt = po.filter_one if impl == "py" else coracle.filter_one
    n_inf = 0
    for i, p, obs, A0, b0 in _cases(F):
        res = flt(p, F["r"][i], obs, F["u0"][i])
        it = int(F["relax_iters"][i])
        if it == 0:
            assert res["status"] == po.STATUS_OPTIMAL, i
        elif it > 0:
            n_inf += 1
            assert res["status"] == po.STATUS_RELAXED and res["iters"] == it, i
        else:
            n_inf += 1
            assert res["status"] == po.STATUS_BOX_INFEASIBLE, i
        assert np.abs(np.asarray(res["x"]) - F["x"][i]).max() <= 1e-12, i
        assert np.abs(np.asarray(res["u"]) - F["u"][i]).max() <= 1e-12, i
    assert n_inf > 100


def test_relaxed_solutions_are_certified(golden):
    """The relaxed minimiser is KKT-certified on the relaxed rows and k is the smallest count."""
    F = golden("golden_filter.npz")
    checked = 0
    for i, p, obs, A0, b0 in _cases(F):
        it = int(F["relax_iters"][i])
        if it <= 0:
            continue
        m = len(obs)
        b = b0.copy(); b[:m] = [po.relaxed_b(v, it) for v in b0[:m]]
        assert qp_bruteforce.kkt_residual(A0, b, F["x"][i]) <= 1e-9
        b1 = b0.copy(); b1[:m] = [po.relaxed_b(v, it - 1) for v in b0[:m]]
        assert qp_bruteforce.solve(A0, b1) is None
        checked += 1
    assert checked > 100


def test_c_matches_python_swarm_bit_exact():
    rng = np.random.default_rng(7)
    for trial in range(12):
        n = int(rng.integers(8, 60)); n_obs = int(rng.integers(0, n // 2))
        pos = rng.uniform(-0.4, 0.4, (n, 2))
        if trial % 3 == 0:
            pos[3] = pos[5]                     # coincident entities
            pos[7] = pos[6] + [0.2, 0.0]        # exactly at the cull radius
        vel = rng.normal(0, 0.3, (n, 2))
        p = po.Params(15)
        c = coracle.filter_swarm(p, pos, vel, n_obs, kmax=64, diag=True)
        u, st, cnt, nbrs = po.filter_swarm(p, pos, vel, n_obs, n_obs, n)
        assert np.array_equal(c["u"], u)
        assert np.array_equal(c["status"], st)
        assert np.array_equal(c["cnt"], cnt)
        for k in range(n - n_obs):
            assert list(c["nbr_idx"][k, :cnt[k]]) == nbrs[k]
            if cnt[k]:
                act, viol = po.diagnose(p, [pos[n_obs + k, 0], pos[n_obs + k, 1], vel[n_obs + k, 0],
                                            vel[n_obs + k, 1]], [[pos[j, 0], pos[j, 1], vel[j, 0], vel[j, 1]]
                                                                 for j in nbrs[k]], vel[n_obs + k], c["x"][k],
                                        st[k] >> 8)
                assert [bool(a) for a in c["nbr_active"][k, :cnt[k]]] == act[:cnt[k]]
                assert [bool(c["box_active"][k] >> b & 1) for b in range(8)] == act[cnt[k]:]
                if st[k] & 0xFF in (po.STATUS_OPTIMAL, po.STATUS_RELAXED):
                    assert c["viol"][k] <= 1e-12


def test_cull_threshold(golden):
    """sqrt(s) < 0.2  <=>  s < 0.04 exactly (cross_and_rescue.py:142-143)."""
    G = golden("golden_cull_threshold.npz")
    t = po.cull_threshold(0.2)
    assert t == 0.04 and t != 0.2 * 0.2
    assert np.array_equal(G["s"] < t, G["keep"])
    for d in (0.2, 0.12, 0.3, 1.0, 0.05):
        t = po.cull_threshold(d)
        s = np.array([np.nextafter(t, 0), t, np.nextafter(t, 1)])
        assert list(np.sqrt(s) < d) == [True, False, False]


def test_consensus_orders(golden):
    """np.sum(X[:,j]-X[:,i,None],1) [@ R * s] for degrees 1..40 (cross_and_rescue.py:118,125)."""
    G = golden("golden_consensus.npz")
    for t in range(len(G["deg"])):
        deg = int(G["deg"][t]); X = G["X"][t][:, :deg + 1].T.copy()
        rp = np.array([0, deg], np.int32); col = np.arange(1, deg + 1, dtype=np.int32)
        th = G["theta"][t]
        plain = coracle.consensus_csr(X, rp, col, 0, deg + 1)
        assert np.array_equal(plain[0], G["plain"][t])
        rot = coracle.consensus_csr(X, rp, col, 0, deg + 1, rot=(np.cos(th), np.sin(th)), scale=G["scale"][t])
        assert np.array_equal(rot[0], G["rot"][t])
        py = po.consensus_csr(X, rp, col, [0], deg + 1, rot=(np.cos(th), np.sin(th)), scale=G["scale"][t])
        assert np.array_equal(py[0], G["rot"][t])


def _car_topology():
    """cross_and_rescue.py:79-95 Laplacians as CSR (topological_neighbors order)."""
    ring = (np.arange(7, dtype=np.int32)[:7], np.array([1, 2, 3, 4, 5, 0], np.int32))
    l2_rows = [[4], [0, 3], [0, 1], [0, 2]]
    rp = np.array([0] + list(np.cumsum([len(r) for r in l2_rows])), np.int32)
    col = np.array(sum(l2_rows, []), np.int32)
    return ring, (rp, col)


@pytest.mark.parametrize("name", ["cross_and_rescue", "meet_at_center", "meet_at_center_n100"])
def test_rollout_steps_vs_golden(golden, name):
    """Per recorded step of the restated caller loops: nominal control, neighbour sets,
    filtered controls and the Euler update, from the golden state at that step."""
    R = golden(f"golden_{name}.npz")
    p = po.Params(15)
    T = 1 / 30
    n_steps = R["pos"].shape[0]
    for t in range(0, n_steps, 1 if name != "meet_at_center_n100" else 3):
        pos, vel = R["pos"][t], R["vel"][t]
        n = pos.shape[0]
        if name == "cross_and_rescue":
            n_obs = 7
            ring = np.array([1, 2, 3, 4, 5, 0], np.int32)
            v_obs = coracle.consensus_csr(pos[:6], np.arange(7, dtype=np.int32), ring, 0, 6,
                                          rot=(np.cos(-np.pi / 6), np.sin(-np.pi / 6)), scale=0.05)
            (_, (rp, col)) = _car_topology()
            v_ag = coracle.consensus_csr(pos[7:], rp, col, 0, 4, anchors=np.array([[1.5, 0.0]]))
            nominal = np.concatenate([v_obs, np.zeros((1, 2)), v_ag])
        else:
            half = n // 2; n_obs = half
            ring = np.array([(i + 1) % half for i in range(half)], np.int32)
            v_obs = coracle.consensus_csr(pos[:half], np.arange(half + 1, dtype=np.int32), ring, 0, half,
                                          rot=(np.cos(-np.pi / half), np.sin(-np.pi / half)))
            rows = [[j for j in range(half) if j != i] for i in range(half)]
            rp = np.array([0] + list(np.cumsum([len(r) for r in rows])), np.int32)
            gain = 1.0 if n == 10 else 4 / 49
            v_ag = coracle.consensus_csr(pos[half:], rp, np.array(sum(rows, []), np.int32), 0, half, scale=gain)
            nominal = np.concatenate([v_obs, v_ag])
        assert np.array_equal(nominal, vel), (name, t)
        out = coracle.filter_swarm(p, pos, vel, n_obs, kmax=n)
        for k in range(n - n_obs):
            got = set(out["nbr_idx"][k, :out["cnt"][k]].tolist())
            assert got == set(np.where(R["nbr_mask"][t][k])[0].tolist()), (name, t, k)
        ref_u = R["u"][t] if R["u"][t].shape[0] == n else np.concatenate([vel[:n_obs], R["u"][t]])
        u = np.concatenate([vel[:n_obs], out["u"]])
        assert np.abs(u - ref_u).max() <= 1e-12, (name, t)
        its = out["status"] >> 8
        assert np.array_equal(np.where(out["cnt"] > 0, its, 0), R["relax_iters"][t]), (name, t)
        nxt = coracle.euler(pos, ref_u, T)
        assert np.array_equal(nxt, R["pos_next"][t]), (name, t)


def test_random_nominal_restatement():
    """oracle random_nominal (numpy uint64) == a pure-Python integer restatement of the hash of
    include/cbf_amd.h CBF_NOMINAL_RANDOM; values lie in [-amp, amp) and change with the position."""
    import struct
    from oracle import pyoracle as po
    M = (1 << 64) - 1

    def mix(z):
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    def bits(v):
        return struct.unpack("<Q", struct.pack("<d", v))[0]

    rng = np.random.default_rng(3)
    pos = rng.normal(size=(200, 2))
    pos[0] = [0.0, -0.0]
    amp, seed, g0 = 1.25, 0xDEADBEEFCAFEF00D, 12345
    got = po.random_nominal(pos, g0, amp, seed)
    for i, (x, y) in enumerate(pos):
        h = mix((seed + 0x9E3779B97F4A7C15 * (g0 + i + 1)) & M)
        h = mix(h ^ bits(x))
        h = mix(h ^ bits(y))
        h2 = mix((h + 0x9E3779B97F4A7C15) & M)
        want = (amp * (2.0 * ((h >> 11) * 2.0 ** -53) - 1.0), amp * (2.0 * ((h2 >> 11) * 2.0 ** -53) - 1.0))
        assert got[i, 0] == want[0] and got[i, 1] == want[1], i
    assert np.all(np.abs(got) <= amp)
    moved = po.random_nominal(pos + 1e-12, g0, amp, seed)
    assert np.all(moved != got)
