"""ctypes binding of libcbf_amd.so (include/cbf_amd.h).

The HIP library is the only compute path: there is no CPU fallback.  Importing this module
fails loudly when the library is missing, and every compute call raises when no ROCm GPU is
visible.  torch supplies device memory and the current HIP stream (plumbing only).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libcbf_amd.so")

CBF_EINVAL = -1
ABI_VERSION = 7  # include/cbf_amd.h CBF_ABI_VERSION
STATUS_IDLE, STATUS_OPTIMAL, STATUS_RELAXED, STATUS_BOX_INFEASIBLE, STATUS_RELAX_CAP = 0, 1, 2, 3, 4
STATUS_NBR_OVERFLOW = 5
STATUS_WORKSPACE_ERROR = 6
RUN_OUTPUT_HISTORY = 1  # cbf_lattice_run_ex flags (include/cbf_amd.h CBF_RUN_*)
RUN_WINDOW_CULL = 2
LAUNCH_SEPARATE_GUARD = 1  # cbf_params.launch_flags (include/cbf_amd.h CBF_LAUNCH_*)
# words of a lattice-step statistics slot (include/cbf_amd.h CBF_STAT_*)
(STAT_SOLVES, STAT_OPTIMAL, STAT_RELAXED, STAT_INFEASIBLE, STAT_SEIDEL, STAT_VIOL_OPTIMAL, STAT_VIOL_ORIGINAL,
 STAT_MIN_DIST2, STAT_ERRORS, STAT_BINDING, STAT_WIN_WALKS, STAT_GUARD_STALLS) = range(12)
_DIST_KEY_TOP = 0x7FF0000000000000


class CbfParams(C.Structure):
    _fields_ = [("max_speed", C.c_double), ("dmin", C.c_double), ("k", C.c_double), ("gamma", C.c_double),
                ("f", C.c_double * 16), ("g", C.c_double * 8), ("cull_t", C.c_double),
                ("nrm", (C.c_double * 2) * 4), ("f_is_zero", C.c_int32), ("relax_cap", C.c_int32),
                ("solve_inline_max", C.c_int32), ("launch_flags", C.c_uint32)]


class CbfGrid(C.Structure):
    _fields_ = [("x0", C.c_double), ("y0", C.c_double), ("inv_h", C.c_double), ("nx", C.c_int32),
                ("ny", C.c_int32)]


class CbfHocbf(C.Structure):
    _fields_ = [("alpha1", C.c_double), ("alpha2", C.c_double)]


class CbfDiag(C.Structure):
    _fields_ = [("kmax", C.c_int32), ("nbr_idx", C.c_void_p), ("nbr_active", C.c_void_p),
                ("box_active", C.c_void_p), ("x", C.c_void_p), ("viol", C.c_void_p)]


class CbfCertParams(C.Structure):
    _fields_ = [("barrier_gain", C.c_double), ("safety_radius", C.c_double), ("magnitude_limit", C.c_double),
                ("boundary_points", C.c_double * 4), ("viol_tol", C.c_double), ("max_iter", C.c_int32)]


class CbfUnicycleParams(C.Structure):
    _fields_ = [("projection_distance", C.c_double), ("angular_velocity_limit", C.c_double),
                ("time_step", C.c_double), ("wheel_radius", C.c_double), ("base_length", C.c_double),
                ("max_linear_velocity", C.c_double), ("max_angular_velocity", C.c_double),
                ("max_wheel_velocity", C.c_double), ("wheel_threshold", C.c_int32)]


CERT_OPTIMAL, CERT_INFEASIBLE, CERT_MAXITER = 1, 2, 3

# symbol -> (restype, argtypes); kept in sync with include/cbf_amd.h (tests check every export)
_vp, _i32, _d, _sz = C.c_void_p, C.c_int32, C.c_double, C.c_size_t
_P, _G, _D = C.POINTER(CbfParams), C.POINTER(CbfGrid), C.POINTER(CbfDiag)
_HP = C.POINTER(CbfHocbf)
_CP, _UP = C.POINTER(CbfCertParams), C.POINTER(CbfUnicycleParams)
SIGNATURES = {
    "cbf_abi_version": (C.c_int, []),
    "cbf_lattice_solves_inline": (C.c_int, [_P, C.c_int64]),  # (include/cbf_amd_measure.h)
    "cbf_workspace_layout": (C.c_int, []),
    "cbf_params_init": (C.c_int, [_P, _d, _d, _d, _vp, _vp, _d]),
    "cbf_get_safe_control_batch": (C.c_int, [_P, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cbf_assemble_rows": (C.c_int, [_P, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cbf_filter_allpairs": (C.c_int, [_P, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _D, _vp]),
    "cbf_cull_allpairs": (C.c_int, [_P, _i32, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "cbf_hocbf_workspace_size": (_sz, [C.c_int64]),
    "cbf_get_safe_control_batch_hocbf": (C.c_int, [_P, _HP, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "cbf_filter_indexed_hocbf": (C.c_int, [_P, _HP, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                           _sz, _vp]),
    "cbf_allpairs_workspace_size": (_sz, [_i32, _i32]),
    "cbf_filter_allpairs_split": (C.c_int, [_P, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _sz, _vp]),
    "cbf_cells_workspace_size": (_sz, [_i32, _G]),
    "cbf_filter_cells": (C.c_int, [_P, _G, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _D, _vp, _sz, _vp]),
    "cbf_consensus_csr": (C.c_int, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _d, _d, _d, _vp, _vp]),
    "cbf_consensus_lattice": (C.c_int, [_i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp]),
    "cbf_euler": (C.c_int, [_i32, _vp, _vp, _d, _vp]),
    "cbf_lattice_workspace_size": (_sz, [_i32, _i32, _G]),
    "cbf_lattice_set_nominal": (C.c_int, [_vp, _sz, _i32, _d, C.c_uint64, _vp]),
    "cbf_lattice_step": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _d, _vp, _vp, _vp, _vp,
                                   _vp, _i32, _vp, _vp, _vp, _sz, _vp]),
    "cbf_lattice_cycle_sharded": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                            _vp, _d, _d,
                                            _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "cbf_lattice_cycle_sharded_ex": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                               _vp, _d, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, C.c_uint32, _vp]),
    "cbf_lattice_run": (C.c_int, [_P, _G, _i32, _i32, _vp, _d, _d, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "cbf_lattice_run_ex": (C.c_int, [_P, _G, _i32, _i32, _vp, _d, _d, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _sz,
                                     C.c_uint32, _vp]),
    "cbf_lattice_workspace_view": (C.c_int64, [_i32, _i32, _G, C.POINTER(C.c_int64)]),
    "cbf_lattice_window_build_ex": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _sz,
                                              _vp]),
    "cbf_lattice_window_advance_ex": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _vp,
                                                _vp, _vp, _vp, _sz, _vp, _vp]),
    "cbf_lattice_window_build": (C.c_int, [_P, _G, _i32, _i32, _vp, _d, _vp, _vp, _sz, _vp]),
    "cbf_lattice_window_counters": (C.c_int, [_vp, _sz, _vp, _vp]),
    "cbf_lattice_window_advance": (C.c_int, [_P, _G, _i32, _i32, _vp, _d, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp,
                                             _vp]),
    "cbf_lattice_build": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _sz, _vp]),
    "cbf_lattice_advance": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _vp, _vp,
                                      _i32, _vp, _vp, _vp, _sz, _vp]),
    "cbf_lattice_advance_marked": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _vp, _vp,
                                      _i32, _vp, _vp, _vp, _sz, _vp, _vp]),
    "cbf_lattice_advance_timed": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _vp, _vp,
                                            _i32, _vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "cbf_lattice_window_advance_timed": (C.c_int, [_P, _G, _i32, _i32, _vp, _d, _vp, _vp, _vp, _vp, _vp, _vp, _sz,
                                                   _vp, _vp, _vp]),
    "cbf_lattice_advance_hocbf": (C.c_int, [_P, _HP, _G, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _vp, _vp, _vp,
                                            _vp, _i32, _vp, _vp, _vp, _sz, _vp]),
    "cbf_mc_rollout": (C.c_int, [_P, _i32, _i32, _i32, _i32, _d, _d, _d, _d, _d, _vp, _vp, _vp, _vp, _vp]),
    "cbf_halo_guard": (C.c_int, [_vp, C.c_int64, _i32, _i32, _d, _vp, _vp]),
    "cbf_halo_ext_bytes": (_sz, [_i32]),
    "cbf_halo_ext_reset": (C.c_int, [_vp, _i32, _vp]),
    "cbf_halo_pack": (C.c_int, [_i32, _i32, C.c_int64, _vp, _vp, _i32, _vp, _vp]),
    "cbf_halo_unpack": (C.c_int, [_i32, _i32, _i32, _i32, C.c_int64, _vp, C.c_int64, _i32, _i32, _d, _i32, _vp, _vp,
                                  _vp]),
    "cbf_halo_nbr_elems": (C.c_int64, [_i32, _i32, _i32, _i32, _i32]),
    "cbf_halo_pack_nbr": (C.c_int, [_i32, _i32, C.c_int64, _vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "cbf_halo_unpack_nbr": (C.c_int, [_i32, _i32, _i32, _i32, C.c_int64, _vp, _i32, _i32, _d, _i32, _vp, _vp,
                                      _vp]),
    "cbf_lattice_step_sharded": (C.c_int, [_P, _G, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _d, _d, _vp,
                                           _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _sz, _vp]),
    "cbf_cert_params_init": (C.c_int, [_CP, _d, _d, _d, _vp]),
    "cbf_si_barrier_cert_lds_bytes": (_sz, [_i32]),
    "cbf_si_barrier_cert": (C.c_int, [_CP, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cbf_unicycle_params_init": (C.c_int, [_UP]),
    "cbf_uni_to_si": (C.c_int, [_UP, _i32, _vp, _vp, _vp]),
    "cbf_unicycle_advance": (C.c_int, [_UP, _i32, _vp, _vp, _vp, _i32, _vp]),
}

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                      "(there is no CPU fallback)")

# torch first: its bundled HIP runtime (soname libamdhip64.so.7) is then the one this library binds
# to.  Loaded the other way round, /opt/rocm's runtime and torch's would both be live in the process
# and torch's device calls fail (hipErrorNoDevice).
import torch  # noqa: E402,F401

lib = C.CDLL(LIB_PATH)
for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args
if lib.cbf_abi_version() != ABI_VERSION:
    raise ImportError(f"{LIB_PATH} has ABI version {lib.cbf_abi_version()}, this package expects {ABI_VERSION}: "
                      "rebuild it")


class CbfError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc == CBF_EINVAL:
        raise CbfError(f"{what}: invalid argument (CBF_EINVAL)")
    if rc != 0:
        raise CbfError(f"{what}: HIP error {rc}")


def make_params(max_speed, dmin=0.2, k=1.0, f=None, g=None, safety_distance=0.2) -> CbfParams:
    p = CbfParams()
    fa = None if f is None else np.ascontiguousarray(np.asarray(f, dtype=np.float64).reshape(16))
    ga = None if g is None else np.ascontiguousarray(np.asarray(g, dtype=np.float64).reshape(8))
    rc = lib.cbf_params_init(C.byref(p), float(max_speed), float(dmin), float(k),
                             None if fa is None else fa.ctypes.data, None if ga is None else ga.ctypes.data,
                             float(safety_distance))
    check(rc, "cbf_params_init")
    return p


def decode_stats(words) -> dict:
    """Host summary of a lattice-step statistics array (uint64[1024] as int64 numpy/torch values:
    64 slots of 16 words, include/cbf_amd.h CBF_STAT_*)."""
    w = np.asarray(words).astype(np.int64).view(np.uint64).reshape(64, 16)
    cnt = {k: int(w[:, i].sum()) for k, i in (("solves", STAT_SOLVES), ("optimal", STAT_OPTIMAL),
                                               ("relaxed", STAT_RELAXED), ("infeasible", STAT_INFEASIBLE),
                                               ("seidel", STAT_SEIDEL), ("errors", STAT_ERRORS),
                                               ("binding", STAT_BINDING), ("win_walks", STAT_WIN_WALKS),
                                               ("guard_stalls", STAT_GUARD_STALLS))}
    vo = w[:, STAT_VIOL_OPTIMAL].max().reshape(1).view(np.float64)[0]
    vr = w[:, STAT_VIOL_ORIGINAL].max().reshape(1).view(np.float64)[0]
    key = int(w[:, STAT_MIN_DIST2].max())
    d2 = None if key == 0 else float(np.array([_DIST_KEY_TOP - key], dtype=np.uint64).view(np.float64)[0])
    cnt.update(viol_optimal=float(vo), viol_original_relaxed=float(vr), min_dist2=d2)
    return cnt


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise CbfError("cbf_amd runs only on a ROCm GPU (MI355X); no GPU is visible and there is no CPU fallback")
    return torch


def stream_handle():
    import torch
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> C.c_void_p:
    return C.c_void_p(0 if t is None else t.data_ptr())
