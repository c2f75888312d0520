"""Drop-in ``ControlBarrierFunction`` (reference cbf.py:5-92) on the MI355X HIP path.

Same constructor, attributes and ``get_safe_control(robot_state, obs_states, f, g, u0)``
signature and return type as the reference; the 2-variable QP is solved exactly on the GPU
(cbf_get_safe_control_batch) instead of by cvxopt.  ``get_safe_control_batch`` is the batched
form for many independent egos with explicit neighbour lists.

``barrier="euclidean_hocbf"`` (keyword-only, not in the reference) swaps the reference's
sign-switched L1 barrier rows (cbf.py:38-59) for Euclidean HOCBF rows of a double integrator,
h = |p_i - p_j|^2 - dmin^2 with psi1 = h' + alpha1 h, psi2 = psi1' + alpha2 psi1 >= 0
(include/cbf_amd.h); f and g are then not used (the dynamics are p' = v, v' = u).
"""
from __future__ import annotations

import threading

import numpy as np

from . import _lib
from ._lib import check, lib, ptr, stream_handle


BARRIERS = ("reference", "euclidean_hocbf")


class ControlBarrierFunction:
    def __init__(self, max_speed, dmin=0.2, k=1, *, barrier="reference", alpha1=1.0, alpha2=1.0):
        """cbf.py:6-16 (barrier / alpha1 / alpha2: the HOCBF mode, see the module docstring)."""
        self.dmin = dmin
        self.k = k
        self.max_speed = max_speed
        self.gamma = 0.5
        if barrier not in BARRIERS:
            raise ValueError(f"barrier must be one of {BARRIERS}, got {barrier!r}")
        self.barrier = barrier
        self.alpha1 = float(alpha1)
        self.alpha2 = float(alpha2)
        # get_safe_control's pinned host / device buffers, one set per device (the call uses the
        # current device's stream); the lock makes the call reentrant across threads sharing one
        # instance, as the stateless reference call is
        self._io = {}
        self._io_lock = threading.Lock()

    def _params(self, f, g):
        f = np.asarray(f, dtype=np.float64)
        g = np.asarray(g, dtype=np.float64)
        if f.shape != (4, 4) or g.shape != (4, 2):
            # the reference's own shape error (cbf.py:55, e.g. its broken __main__ demo)
            raise ValueError(f"f must be 4x4 and g 4x2 for the [x, y, vx, vy] state, got {f.shape} and {g.shape}")
        p = _lib.make_params(self.max_speed, self.dmin, self.k, f, g)
        p.gamma = float(self.gamma)
        return p

    def get_safe_control(self, robot_state, obs_states, f, g, u0):
        """cbf.py:18-92: barrier rows per obstacle, 8 box rows, min |x|^2 s.t. Ax <= b, then
        u = clip(x + u0, +-max_speed).  Returns a float64 ndarray of shape (2,)."""
        torch = _lib.require_gpu()
        r = np.asarray(robot_state, dtype=np.float64).reshape(4)
        obs = np.asarray(obs_states, dtype=np.float64).reshape(-1, 4)
        u0 = np.asarray(u0, dtype=np.float64).reshape(2)
        m = obs.shape[0]
        # one pinned host buffer, one copy to the device: [state (4), u0 (2), obstacles (4 m, at
        # least 4)] as float64, then the neighbour offsets {0, m} as int32 in the last 8 bytes.
        # The buffers are kept per instance and device and grown as needed; every call ends
        # synchronised (the result is read back) before the lock is released, so the next call
        # may overwrite them.
        nf = 6 + 4 * max(m, 1)
        nbytes = 8 * nf + 8
        dev = torch.cuda.current_device()
        with self._io_lock:
            io = self._io.get(dev)
            if io is None or io[0].numel() < nbytes:
                cap = max(nbytes, 8 * (6 + 4 * 64) + 8)
                io = (torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                      torch.empty(cap, dtype=torch.uint8, device=f"cuda:{dev}"),
                      torch.empty(2, dtype=torch.float64, pin_memory=True))
                self._io[dev] = io
            pin, dev_buf, out = io
            host = pin.numpy()
            hf = host[:8 * nf].view(np.float64)
            hf[:4] = r
            hf[4:6] = u0
            hf[6:6 + 4 * m] = obs.reshape(-1)
            if m == 0:
                hf[6:10] = 0.0
            host[8 * nf:nbytes].view(np.int32)[:] = (0, m)
            dev_buf[:nbytes].copy_(pin[:nbytes], non_blocking=True)
            df = dev_buf[:8 * nf].view(torch.float64)
            off = dev_buf[8 * nf:nbytes].view(torch.int32)
            u, _, _ = self.get_safe_control_batch(df[:4].view(1, 4), (off, df[6:].view(-1, 4)), df[4:6].view(1, 2),
                                                  f, g)
            out.copy_(u[0], non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return out.numpy().copy()

    def get_safe_control_batch(self, robot_states, obs_list, u0, f=None, g=None, return_x=False):
        """Batched get_safe_control.  robot_states (B,4), u0 (B,2) float64 CUDA tensors; obs_list is
        either a list of B (m_i,4) tensors or a tuple (nbr_off int32 (B+1,), obs_states (M,4)).
        Returns (u (B,2), status int32 (B,), x (B,2) or None)."""
        torch = _lib.require_gpu()
        f = np.zeros((4, 4)) if f is None else f
        g = 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]]) if g is None else g
        p = self._params(f, g)
        dev = robot_states.device
        B = robot_states.shape[0]
        if isinstance(obs_list, tuple):
            off, obs = obs_list
        else:
            counts = [int(o.shape[0]) for o in obs_list]
            off = torch.tensor(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32), device=dev)
            obs = torch.cat([o.reshape(-1, 4) for o in obs_list]) if counts and sum(counts) else \
                torch.zeros((1, 4), dtype=torch.float64, device=dev)
        rs = robot_states.contiguous().to(torch.float64)
        u0 = u0.contiguous().to(torch.float64)
        obs = obs.contiguous().to(torch.float64)
        off = off.contiguous().to(torch.int32)
        assert rs.shape == (B, 4) and u0.shape == (B, 2) and off.shape == (B + 1,)
        u = torch.empty((B, 2), dtype=torch.float64, device=dev)
        st = torch.empty((B,), dtype=torch.int32, device=dev)
        x = torch.empty((B, 2), dtype=torch.float64, device=dev) if return_x else None
        if self.barrier == "euclidean_hocbf":
            rows = int(off[-1].item())
            need = lib.cbf_hocbf_workspace_size(rows)
            ws = torch.empty((need,), dtype=torch.uint8, device=dev)
            hp = _lib.CbfHocbf(self.alpha1, self.alpha2)
            check(lib.cbf_get_safe_control_batch_hocbf(p, _lib.C.byref(hp), B, ptr(rs), ptr(u0), ptr(off), ptr(obs),
                                                       ptr(u), ptr(st), ptr(x), ptr(ws), need, stream_handle()),
                  "cbf_get_safe_control_batch_hocbf")
            return u, st, x
        check(lib.cbf_get_safe_control_batch(p, B, ptr(rs), ptr(u0), ptr(off), ptr(obs), ptr(u), ptr(st), ptr(x),
                                             stream_handle()), "cbf_get_safe_control_batch")
        return u, st, x

    def assemble_rows(self, robot_states, nbr_off, obs_states, u0, f=None, g=None):
        """(A, b) exactly as cbf.py:72-80 hands them to cvxopt, for a batch (rows of ego i at
        [off[i] + 8 i, off[i+1] + 8 (i+1)))."""
        torch = _lib.require_gpu()
        f = np.zeros((4, 4)) if f is None else f
        g = 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]]) if g is None else g
        p = self._params(f, g)
        B = robot_states.shape[0]
        M = int(nbr_off[-1].item())
        dev = robot_states.device
        A = torch.empty((M + 8 * B, 2), dtype=torch.float64, device=dev)
        b = torch.empty((M + 8 * B,), dtype=torch.float64, device=dev)
        check(lib.cbf_assemble_rows(p, B, ptr(robot_states.contiguous()), ptr(u0.contiguous()),
                                    ptr(nbr_off.contiguous()), ptr(obs_states.contiguous()), ptr(A), ptr(b),
                                    stream_handle()), "cbf_assemble_rows")
        return A, b
