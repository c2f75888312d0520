"""ctypes wrapper for the C oracle (oracle/cbf_oracle.c).

TEST INFRASTRUCTURE ONLY -- the checker for tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  Numpy arrays in, numpy arrays out.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc.so")


class OrcParams(C.Structure):
    _fields_ = [("max_speed", C.c_double), ("dmin", C.c_double), ("k", C.c_double), ("gamma", C.c_double),
                ("f", C.c_double * 16), ("g", C.c_double * 8), ("cull_t", C.c_double)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp, ip, i64p, u8p = (np.ctypeslib.ndpointer(np.float64, flags="C"),
                             np.ctypeslib.ndpointer(np.int32, flags="C"),
                             np.ctypeslib.ndpointer(np.int64, flags="C"),
                             np.ctypeslib.ndpointer(np.uint8, flags="C"))
        P = C.POINTER(OrcParams)
        L.orc_assemble.argtypes = [P, dp, C.c_int, dp, dp, dp, dp]
        L.orc_filter_one.argtypes = [P, dp, C.c_int, dp, dp, dp, dp, C.POINTER(C.c_int)]
        L.orc_filter_one.restype = C.c_int
        L.orc_filter_swarm.argtypes = [P, C.c_int, C.c_int, dp, dp, C.c_int, C.c_int, dp, ip, ip,
                                       C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
        L.orc_consensus_csr.argtypes = [C.c_int, C.c_int, C.c_int, dp, C.c_void_p, ip, ip, C.c_int, C.c_double,
                                        C.c_double, C.c_double, dp]
        L.orc_consensus_lattice.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, C.c_double, dp]
        L.orc_euler.argtypes = [C.c_int, dp, dp, C.c_double]
        L.orc_mc_rollout.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                     C.c_double, C.c_double, dp, i64p, dp, C.c_void_p]
        L.orc_filter_one_hocbf.argtypes = [P, C.c_double, C.c_double, dp, C.c_int, dp, dp, dp, dp,
                                           C.POINTER(C.c_int)]
        L.orc_filter_one_hocbf.restype = C.c_int
        L.orc_filter_swarm_hocbf.argtypes = [P, C.c_double, C.c_double, C.c_int, C.c_int, dp, dp, C.c_int, C.c_int,
                                             dp, ip, ip, C.c_void_p]
        _lib = L
    return _lib


def params(p) -> OrcParams:
    """From any object with max_speed, dmin, k, gamma, f(4x4), g(4x2), cull_t."""
    o = OrcParams()
    o.max_speed, o.dmin, o.k, o.gamma = float(p.max_speed), float(p.dmin), float(p.k), float(p.gamma)
    o.f[:] = [float(v) for v in np.asarray(p.f, dtype=np.float64).reshape(16)]
    o.g[:] = [float(v) for v in np.asarray(p.g, dtype=np.float64).reshape(8)]
    o.cull_t = float(p.cull_t)
    return o


def _c(a, dt=np.float64):
    return np.ascontiguousarray(a, dtype=dt)


def assemble(p, r, obs, u0):
    obs = _c(obs).reshape(-1, 4)
    m = obs.shape[0]
    A = np.zeros((m + 8, 2)); b = np.zeros(m + 8)
    lib().orc_assemble(C.byref(params(p)), _c(r), m, obs, _c(u0), A, b)
    return A, b


def filter_one(p, r, obs, u0):
    obs = _c(obs).reshape(-1, 4)
    u = np.zeros(2); x = np.zeros(2); it = C.c_int(0)
    st = lib().orc_filter_one(C.byref(params(p)), _c(r), obs.shape[0], obs, _c(u0), u, x, C.byref(it))
    return dict(u=u, x=x, status=st, iters=it.value)


def filter_swarm(p, pos, vel, n_obs, ego_begin=None, ego_end=None, kmax=0, diag=False, stats=False):
    """cross_and_rescue.py:135-160 for egos [ego_begin, ego_end).  diag: neighbour indices / active
    flags, box bits, x, viol (solved rows); stats: viol_orig (original rows) and d2min (smallest
    neighbour distance^2, +inf if none)."""
    pos = _c(pos).reshape(-1, 2); vel = _c(vel).reshape(-1, 2)
    n = pos.shape[0]
    eb = n_obs if ego_begin is None else ego_begin
    ee = n if ego_end is None else ego_end
    ne = ee - eb
    u = np.zeros((ne, 2)); st = np.zeros(ne, np.int32); cnt = np.zeros(ne, np.int32)
    out = dict(u=u, status=st, cnt=cnt)
    ptrs = [None] * 7
    if kmax:
        out["nbr_idx"] = np.zeros((ne, kmax), np.int32)
        ptrs[0] = out["nbr_idx"].ctypes.data
        if diag:
            out["nbr_active"] = np.zeros((ne, kmax), np.uint8)
            ptrs[1] = out["nbr_active"].ctypes.data
    if diag:
        out["box_active"] = np.zeros(ne, np.uint8); ptrs[2] = out["box_active"].ctypes.data
        out["x"] = np.zeros((ne, 2)); ptrs[3] = out["x"].ctypes.data
        out["viol"] = np.zeros(ne); ptrs[4] = out["viol"].ctypes.data
    if stats:
        out["viol_orig"] = np.zeros(ne); ptrs[5] = out["viol_orig"].ctypes.data
        out["d2min"] = np.zeros(ne); ptrs[6] = out["d2min"].ctypes.data
    lib().orc_filter_swarm(C.byref(params(p)), n, n_obs, pos, vel, eb, ee, u, st, cnt, ptrs[0], ptrs[1], kmax,
                           ptrs[2], ptrs[3], ptrs[4], ptrs[5], ptrs[6])
    return out


def consensus_csr(src, row_ptr, col, self_offset, n_group, anchors=None, rot=None, scale=1.0):
    src = _c(src).reshape(-1, 2)
    row_ptr = _c(row_ptr, np.int32); col = _c(col, np.int32)
    n_dst = len(row_ptr) - 1
    out = np.zeros((n_dst, 2))
    anc = None if anchors is None else _c(anchors).reshape(-1, 2)
    rc, rs = (1.0, 0.0) if rot is None else rot
    lib().orc_consensus_csr(n_dst, self_offset, n_group, src, None if anc is None else anc.ctypes.data,
                            row_ptr, col, 0 if rot is None else 1, rc, rs, scale, out)
    return out


def consensus_lattice(W, H, row_begin, row_end, pos, scale):
    pos = _c(pos).reshape(-1, 2)
    out = np.zeros(((row_end - row_begin) * W, 2))
    lib().orc_consensus_lattice(W, H, row_begin, row_end, pos, scale, out)
    return out


def euler(pos, vel, T):
    pos = _c(pos).copy().reshape(-1, 2)
    lib().orc_euler(pos.shape[0], pos, _c(vel).reshape(-1, 2), T)
    return pos


def mc_rollout(p, pos, n_o, n_a, steps, T, rot, so, ga, safety=False):
    """Returns (pos, counters, maxviol[, safety (n_scen, 2) = {max original-row violation over
    RELAXED solves, min neighbour distance^2}])."""
    pos = _c(pos).copy()
    n_scen = pos.shape[0]
    counters = np.zeros((n_scen, 4), np.int64); mv = np.zeros(n_scen)
    sf = np.zeros((n_scen, 2)) if safety else None
    lib().orc_mc_rollout(C.byref(params(p)), n_scen, n_o, n_a, steps, T, rot[0], rot[1], so, ga, pos, counters, mv,
                         None if sf is None else sf.ctypes.data)
    return (pos, counters, mv, sf) if safety else (pos, counters, mv)


def filter_one_hocbf(p, hp, r, obs, u0):
    """Euclidean HOCBF mode (pyoracle.filter_one_hocbf) in C."""
    obs = _c(obs).reshape(-1, 4)
    u = np.zeros(2); x = np.zeros(2); it = C.c_int(0)
    st = lib().orc_filter_one_hocbf(C.byref(params(p)), hp.a_sum, hp.a_prod, _c(r), obs.shape[0], obs, _c(u0), u, x,
                                    C.byref(it))
    return dict(u=u, x=x, status=st, iters=it.value)


def filter_swarm_hocbf(p, hp, pos, vel, n_obs, ego_begin=None, ego_end=None):
    pos = _c(pos).reshape(-1, 2); vel = _c(vel).reshape(-1, 2)
    n = pos.shape[0]
    eb = n_obs if ego_begin is None else ego_begin
    ee = n if ego_end is None else ego_end
    ne = ee - eb
    u = np.zeros((ne, 2)); st = np.zeros(ne, np.int32); cnt = np.zeros(ne, np.int32); x = np.zeros((ne, 2))
    lib().orc_filter_swarm_hocbf(C.byref(params(p)), hp.a_sum, hp.a_prod, n, n_obs, pos, vel, eb, ee, u, st, cnt,
                                 x.ctypes.data)
    return dict(u=u, status=st, cnt=cnt, x=x)
