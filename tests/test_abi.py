"""C-ABI library: loads, exports every symbol include/cbf_amd.h declares, host-side parameter
setup matches the oracle, and argument validation rejects bad calls before any launch.
CPU only (no compute calls)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle import pyoracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


HEADERS = ("cbf_amd.h", "cbf_amd_measure.h")  # the drop-in surface; the bench's measurement hooks


def _declared(headers=HEADERS):
    names = set()
    for h in headers:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:int|int64_t|size_t)\s+(cbf_\w+)\s*\(", src, flags=re.M))
    return sorted(names)


def test_measurement_hooks_are_not_in_the_public_header():
    public, hooks = set(_declared(("cbf_amd.h",))), set(_declared(("cbf_amd_measure.h",)))
    assert hooks == {"cbf_lattice_advance_marked", "cbf_lattice_advance_timed", "cbf_lattice_window_advance_timed",
                     "cbf_lattice_solves_inline"}
    assert not public & hooks


def test_solves_inline_query_follows_the_params():
    from cbf_amd import _lib, swarm
    for placement, n, want in (("inline", 1 << 30, 1), ("queued", 16, 0), (4096, 4096, 1), (4096, 4097, 0)):
        cp = swarm.FilterParams(solve_placement=placement).c()
        assert _lib.lib.cbf_lattice_solves_inline(C.byref(cp), n) == want, (placement, n)
    cp = swarm.FilterParams().c()   # "auto": the library's threshold, inline for small windows only
    assert _lib.lib.cbf_lattice_solves_inline(C.byref(cp), 1024) == 1
    assert _lib.lib.cbf_lattice_solves_inline(C.byref(cp), 1 << 20) == 0


def test_library_loads_and_exports_every_declared_symbol():
    from cbf_amd import _lib
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(_lib.lib, n), n
        assert n in _lib.SIGNATURES, n
    assert set(_lib.SIGNATURES) == set(names)
    assert _lib.lib.cbf_abi_version() == _lib.ABI_VERSION == 7


def test_library_is_gfx950_code_object():
    from cbf_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("k", [1, 2, 0.5, 3])
def test_params_init_matches_oracle(k):
    from cbf_amd import _lib
    rng = np.random.default_rng(int(k * 10))
    for trial in range(20):
        g = None if trial == 0 else rng.normal(0, 0.3, (4, 2))
        f = None if trial < 10 else rng.normal(0, 0.1, (4, 4))
        d = float(rng.choice([0.2, 0.12, 0.3]))
        cp = _lib.make_params(15, 0.2, k, f, g, d)
        pp = po.Params(15, 0.2, k, f=f, g=g, safety_distance=d)
        assert cp.cull_t == pp.cull_t
        assert cp.gamma == 0.5 and cp.relax_cap == 1 << 16
        assert cp.f_is_zero == (1 if f is None else 0)
        for q in range(4):
            assert tuple(cp.nrm[q]) == po.quadrant_normal(pp, q)
    cp = _lib.make_params(15)
    assert cp.cull_t == 0.04 and list(cp.g) == [0.1, 0, 0, 0.1, 0, 0, 0, 0]


def test_argument_validation_without_launch():
    from cbf_amd import _lib
    L = _lib.lib
    cp = _lib.make_params(15)
    null = None
    # n_obs > n
    assert L.cbf_filter_allpairs(cp, 4, 5, 1, 1, 5, 4, 1, 1, null, null, null) == _lib.CBF_EINVAL
    # ego range outside the agents
    assert L.cbf_filter_allpairs(cp, 10, 5, 1, 1, 2, 10, 1, 1, null, null, null) == _lib.CBF_EINVAL
    # cell edge below the cull radius
    g = _lib.CbfGrid(); g.x0 = g.y0 = 0.0; g.inv_h = 10.0; g.nx = g.ny = 4
    assert L.cbf_filter_cells(cp, C.byref(g), 8, 0, 1, 1, 0, 8, 1, 1, null, null, 1, 1 << 20,
                              null) == _lib.CBF_EINVAL
    # lattice window missing the neighbour row
    g.inv_h = 4.0
    assert L.cbf_lattice_step(cp, C.byref(g), 8, 8, 2, 4, 2, 2, 1, 0.25, 0.1, 1, 1, 1, 1, null, 0, null, null, 1,
                              1 << 24, null) == _lib.CBF_EINVAL
    # multi-timestep run: negative step count; window too large for 32-bit slot offsets
    assert L.cbf_lattice_run(cp, C.byref(g), 8, 8, 1, 0.25, 0.1, -1, 1, 1, 1, null, null, 1, 1 << 24,
                             null) == _lib.CBF_EINVAL
    assert L.cbf_lattice_run(cp, C.byref(g), 1 << 14, 1 << 14, 1, 0.25, 0.1, 1, 1, 1, 1, null, null, 1, 1 << 62,
                             null) == _lib.CBF_EINVAL
    # mc: too many entities per scenario
    assert L.cbf_mc_rollout(cp, 4, 200, 100, 1, 0.1, 1.0, 0.0, 1.0, 1.0, 1, 1, 1, null, null) == _lib.CBF_EINVAL
    # sharded halo exchange: bad geometry is refused before any launch
    assert L.cbf_halo_ext_bytes(0) == 0 and L.cbf_halo_ext_bytes(4) == 4 * L.cbf_halo_ext_bytes(1)
    assert L.cbf_halo_pack(8, 4, 16, 1, 1, 1, 1, null) == _lib.CBF_EINVAL          # fewer owned rows than 2 halos
    assert L.cbf_halo_pack(8, 2, 64, 1, 1, 0, 1, null) == _lib.CBF_EINVAL          # no sub-step records
    assert L.cbf_halo_unpack(8, 2, 2, 0, 0, 1, 4 * 2 * 8 + 8, 2, 0, 0.2, 1, 1, 1, null) == _lib.CBF_EINVAL  # rank 0 below
    assert L.cbf_halo_unpack(8, 2, 0, 2, 2, 1, 4 * 2 * 8, 2, 0, 0.2, 1, 1, 1, null) == _lib.CBF_EINVAL      # stride short
    # neighbour exchange: buffer sizes (records to every rank, rows to the two neighbours only)
    assert L.cbf_halo_nbr_elems(8, 2, 3, 1, 0) == 24                          # one rank: its own records
    assert L.cbf_halo_nbr_elems(8, 2, 3, 4, 0) == 4 * 24 + 2 * 2 * 8          # an edge rank: one neighbour
    assert L.cbf_halo_nbr_elems(8, 2, 3, 4, 2) == 4 * 24 + 2 * 2 * 2 * 8      # a middle rank: two
    assert L.cbf_halo_nbr_elems(8, 2, 3, 4, 4) == -1
    assert L.cbf_halo_pack_nbr(8, 2, 64, 1, 1, 1, 2, 2, 1, null) == _lib.CBF_EINVAL      # rank outside the world
    assert L.cbf_halo_pack_nbr(8, 4, 16, 1, 1, 1, 2, 0, 1, null) == _lib.CBF_EINVAL      # fewer owned rows than 2 halos
    assert L.cbf_halo_unpack_nbr(8, 2, 2, 0, 0, 1, 2, 0, 0.2, 1, 1, 1, null) == _lib.CBF_EINVAL  # rank 0 has no rows below
    assert L.cbf_halo_unpack_nbr(8, 2, 0, 2, 2, 1, 2, 1, 0.2, 1, 1, 1, null) == _lib.CBF_EINVAL  # last rank none above
    assert L.cbf_lattice_step_sharded(cp, C.byref(g), 8, 8, 0, 8, 2, 9, 0, 8, 1, 0.25, 0.1, 1, 1, 1, 1, null, 3, 1,
                                      null, 1, 1 << 24, null) == _lib.CBF_EINVAL   # owned rows outside the computed rows
    # certificate / unicycle
    cc = _lib.CbfCertParams()
    assert L.cbf_cert_params_init(C.byref(cc), 100.0, 0.12, 0.2, null) == 0 and list(cc.boundary_points) == [-1.6, 1.6,
                                                                                                               -1.0, 1.0]
    assert L.cbf_si_barrier_cert(C.byref(cc), 4, 33, 1, 1, 1, 1, null, null, null) == _lib.CBF_EINVAL   # > 32 agents
    assert L.cbf_si_barrier_cert_lds_bytes(16) > 0 and L.cbf_si_barrier_cert_lds_bytes(33) == 0
    uu = _lib.CbfUnicycleParams()
    assert L.cbf_unicycle_params_init(C.byref(uu)) == 0 and uu.max_wheel_velocity == 12.5
    assert L.cbf_unicycle_advance(C.byref(uu), 4, 1, 1, null, 1, null) == _lib.CBF_EINVAL   # mode 1 needs dxu
    assert L.cbf_unicycle_advance(C.byref(uu), 4, 1, 1, 1, 3, null) == _lib.CBF_EINVAL      # no mode 3
    # zero-size calls are no-ops
    assert L.cbf_euler(0, null, null, 0.1, null) == 0
    assert L.cbf_si_barrier_cert(C.byref(cc), 0, 4, null, null, null, null, null, null, null) == 0
    assert L.cbf_get_safe_control_batch(cp, 0, null, null, null, null, null, null, null, null) == 0


def test_decode_stats():
    """Host decoding of the lattice-step statistics words (include/cbf_amd.h CBF_STAT_*)."""
    from cbf_amd import _lib
    w = np.zeros(1024, np.uint64)
    assert _lib.decode_stats(w.view(np.int64)) == {"solves": 0, "optimal": 0, "relaxed": 0, "infeasible": 0,
                                                   "seidel": 0, "errors": 0, "binding": 0, "win_walks": 0,
                                                   "guard_stalls": 0, "viol_optimal": 0.0,
                                                   "viol_original_relaxed": 0.0, "min_dist2": None}
    s = w.reshape(64, 16)
    s[3, _lib.STAT_SOLVES] = 5
    s[60, _lib.STAT_SOLVES] = 7
    s[1, _lib.STAT_OPTIMAL] = 4
    s[2, _lib.STAT_VIOL_OPTIMAL] = np.array([1e-17]).view(np.uint64)[0]
    s[9, _lib.STAT_VIOL_OPTIMAL] = np.array([3e-18]).view(np.uint64)[0]
    s[4, _lib.STAT_VIOL_ORIGINAL] = np.array([0.25]).view(np.uint64)[0]
    for slot, d2 in ((5, 0.01), (6, 0.0049), (7, 0.03)):
        s[slot, _lib.STAT_MIN_DIST2] = np.uint64(0x7FF0000000000000) - np.array([d2]).view(np.uint64)[0]
    s[11, _lib.STAT_WIN_WALKS] = 9
    s[12, _lib.STAT_GUARD_STALLS] = 2
    d = _lib.decode_stats(w.view(np.int64))
    assert d["solves"] == 12 and d["optimal"] == 4 and d["win_walks"] == 9 and d["guard_stalls"] == 2
    assert d["viol_optimal"] == 1e-17 and d["viol_original_relaxed"] == 0.25 and d["min_dist2"] == 0.0049


def test_workspace_sizes():
    from cbf_amd import _lib, swarm
    g = swarm.make_grid(-1, -1, 150, 150, 0.204)
    n = 1 << 20
    ws = _lib.lib.cbf_lattice_workspace_size(1024, 1024, C.byref(g))
    cells = _lib.lib.cbf_cells_workspace_size(n, C.byref(g))
    assert cells > 60 * n and ws > cells
    assert ws < 200 * n   # stays well inside 288 GB HBM even at 1e9 agents / 8 GPUs


def test_product_path_has_no_cpu_fallback():
    """The package never imports the oracle, and compute calls refuse to run without a GPU."""
    import cbf_amd
    pkg = os.path.dirname(cbf_amd.__file__)
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            txt = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in re.sub(r'""".*?"""|#.*', "", txt, flags=re.S), fn
    import torch
    if not torch.cuda.is_available():
        with pytest.raises(cbf_amd.CbfError):
            cbf_amd.ControlBarrierFunction(15).get_safe_control(np.zeros(4), np.zeros((1, 4)), np.zeros((4, 4)),
                                                                0.1 * np.eye(4, 2), [0.0, 0.0])


def test_torch_extension_registers_ops():
    """The thin PyTorch-ROCm extension (torch.ops.cbf_amd, csrc/torch_ops.cpp) loads, exposes the
    reference call surface over the C ABI, and has no CPU kernels (no fallback)."""
    import torch
    from cbf_amd import _lib, swarm, torch_ops
    o = torch_ops.ops()
    for name in ("get_safe_control_batch", "filter_swarm", "lattice_step", "lattice_run", "lattice_workspace_size",
                 "abi_version"):
        assert hasattr(o, name), name
    assert o.abi_version() == _lib.ABI_VERSION
    g = swarm.make_grid(-1.0, -1.0, 20.0, 30.0, 0.204)
    assert o.lattice_workspace_size(96, 128, g.x0, g.y0, 1 / g.inv_h, g.nx, g.ny) == \
        _lib.lib.cbf_lattice_workspace_size(96, 128, C.byref(g))
    with pytest.raises((NotImplementedError, RuntimeError)):
        o.filter_swarm(torch.zeros(4, 2, dtype=torch.float64), torch.zeros(4, 2, dtype=torch.float64), 0, 15.0)
