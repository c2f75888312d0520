"""robotarium-lite: the rps calls the reference scripts wrap around the filter, on the GPU.

SURVEY.md 8(f) rows 2-3.  The reference scripts import robotarium_python_simulator (``rps``;
/root/reference/install.sh:1 clones it at an unpinned HEAD, absent from this image) for

* ``create_si_to_uni_mapping()``  -> ``si_to_uni_dyn``, ``uni_to_si_states``
  (cross_and_rescue.py:75,101,167; meet_at_center.py:61,80,148)
* ``create_single_integrator_barrier_certificate_with_boundary(safety_radius=0.12)``
  (cross_and_rescue.py:72,163; meet_at_center.py:58, applied only in a comment at :109)
* ``Robotarium.get_poses / set_velocities / step`` (cross_and_rescue.py:100,170,175)

This module keeps those call surfaces (numpy ``(2, N)`` / ``(3, N)`` arrays in and out) and
runs them through the HIP library (``rps.hip``): the coupled barrier-certificate QP is solved
exactly (Goldfarb-Idnani, one wavefront per scenario), batched over independent scenarios
with ``SiBarrierCert.batch``.  ``CrossAndRescue`` runs cross_and_rescue.py's whole loop as
shipped (unicycle robots + the CBF filter + the certificate) device-resident.  Parity against
rps itself is unpinned; tests compare with the restatement in oracle/rps_lite.py.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import CbfCertParams, CbfUnicycleParams, check, lib, ptr, stream_handle
from .swarm import FilterParams, consensus_csr, csr_from_rows, euler, filter_swarm


def _dev_tensor(a, torch, dev, cols):
    """(cols, N) numpy (rps layout) or (N, cols) CUDA tensor -> contiguous (N, cols) CUDA tensor."""
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=torch.float64).contiguous()
    a = np.asarray(a, dtype=np.float64)
    if a.ndim != 2 or a.shape[0] != cols:
        raise ValueError(f"expected a ({cols}, N) array, got shape {a.shape}")
    return torch.tensor(np.ascontiguousarray(a.T), device=dev)


def unicycle_params(projection_distance=0.05, angular_velocity_limit=np.pi, wheel_threshold=True) -> CbfUnicycleParams:
    u = CbfUnicycleParams()
    check(lib.cbf_unicycle_params_init(C.byref(u)), "cbf_unicycle_params_init")
    u.projection_distance = float(projection_distance)
    u.angular_velocity_limit = float(angular_velocity_limit)
    u.wheel_threshold = 1 if wheel_threshold else 0
    return u


def uni_to_si(u: CbfUnicycleParams, poses, out=None):
    """(N, 3) CUDA poses -> (N, 2) projection points (uni_to_si_states)."""
    torch = _lib.require_gpu()
    n = poses.shape[0]
    if out is None:
        out = torch.empty((n, 2), dtype=torch.float64, device=poses.device)
    check(lib.cbf_uni_to_si(C.byref(u), n, ptr(poses), ptr(out), stream_handle()), "cbf_uni_to_si")
    return out


def unicycle_advance(u: CbfUnicycleParams, poses, dxi, mode=0, dxu=None):
    """mode 0: poses <- step(set_velocities(si_to_uni_dyn(dxi, poses))) in place; mode 1:
    dxu = si_to_uni_dyn(dxi, poses); mode 2: dxi holds (v, w), poses <- step(set_velocities(dxi))."""
    torch = _lib.require_gpu()
    n = poses.shape[0]
    if mode == 1 and dxu is None:
        dxu = torch.empty((n, 2), dtype=torch.float64, device=poses.device)
    check(lib.cbf_unicycle_advance(C.byref(u), n, ptr(poses), ptr(dxi.contiguous()), ptr(dxu), int(mode),
                                   stream_handle()), "cbf_unicycle_advance")
    return dxu


def create_si_to_uni_mapping(projection_distance=0.05, angular_velocity_limit=np.pi):
    """rps.utilities.transformations.create_si_to_uni_mapping: returns (si_to_uni_dyn,
    uni_to_si_states) taking and returning rps-layout numpy arrays (cross_and_rescue.py:75)."""
    torch = _lib.require_gpu()
    dev = torch.device("cuda")
    u = unicycle_params(projection_distance, angular_velocity_limit)

    def si_to_uni_dyn(dxi, poses):
        p = _dev_tensor(poses, torch, dev, 3)
        d = _dev_tensor(dxi, torch, dev, 2)
        return unicycle_advance(u, p, d, mode=1).cpu().numpy().T.copy()

    def uni_to_si_states(poses):
        return uni_to_si(u, _dev_tensor(poses, torch, dev, 3)).cpu().numpy().T.copy()

    return si_to_uni_dyn, uni_to_si_states


class SiBarrierCert:
    """rps create_single_integrator_barrier_certificate_with_boundary(...): ``f(dxi, x)`` maps
    (2, N) velocities at (2, N) positions to the exact minimiser of the certificate QP
    (rps solves it with cvxopt); ``batch`` runs independent scenarios (B, N, 2) on the GPU.
    Unlike rps, the caller's dxi is not thresholded in place."""

    MAX_AGENTS = 32

    def __init__(self, barrier_gain=100, safety_radius=0.17, magnitude_limit=0.2,
                 boundary_points=(-1.6, 1.6, -1.0, 1.0)):
        self.c = CbfCertParams()
        bp = np.ascontiguousarray(np.asarray(boundary_points, dtype=np.float64).reshape(4))
        check(lib.cbf_cert_params_init(C.byref(self.c), float(barrier_gain), float(safety_radius),
                                       float(magnitude_limit), bp.ctypes.data), "cbf_cert_params_init")

    def batch(self, dxi, x, iters=False):
        """dxi, x: (B, N, 2) float64 CUDA tensors -> dict(out (B, N, 2), status (B,) [, iters, n_active])."""
        torch = _lib.require_gpu()
        if dxi.dim() != 3 or dxi.shape != x.shape or dxi.shape[2] != 2:
            raise ValueError(f"dxi and x must both be (B, N, 2), got {tuple(dxi.shape)} and {tuple(x.shape)}")
        B, N = dxi.shape[0], dxi.shape[1]
        if not 1 <= N <= self.MAX_AGENTS:
            raise _lib.CbfError(f"si_barrier_cert: 1 <= N <= {self.MAX_AGENTS} agents per scenario, got {N}")
        dev = dxi.device
        res = {"out": torch.empty((B, N, 2), dtype=torch.float64, device=dev),
               "status": torch.empty((B,), dtype=torch.int32, device=dev)}
        if iters:
            res["iters"] = torch.empty((B,), dtype=torch.int32, device=dev)
            res["n_active"] = torch.empty((B,), dtype=torch.int32, device=dev)
        check(lib.cbf_si_barrier_cert(C.byref(self.c), B, N, ptr(dxi.contiguous()), ptr(x.contiguous()),
                                      ptr(res["out"]), ptr(res["status"]), ptr(res.get("iters")),
                                      ptr(res.get("n_active")), stream_handle()), "cbf_si_barrier_cert")
        return res

    def __call__(self, dxi, x):
        torch = _lib.require_gpu()
        dev = torch.device("cuda")
        d = _dev_tensor(dxi, torch, dev, 2)
        p = _dev_tensor(x, torch, dev, 2)
        if d.shape != p.shape:
            raise ValueError(f"dxi and x shapes differ: {tuple(d.shape)} vs {tuple(p.shape)}")
        r = self.batch(d[None], p[None])
        return r["out"][0].cpu().numpy().T.copy()


def create_single_integrator_barrier_certificate_with_boundary(barrier_gain=100, safety_radius=0.17,
                                                               magnitude_limit=0.2,
                                                               boundary_points=np.array([-1.6, 1.6, -1.0, 1.0])):
    """rps.utilities.barrier_certificates entry point (cross_and_rescue.py:72)."""
    return SiBarrierCert(barrier_gain, safety_radius, magnitude_limit, boundary_points)


class Robotarium:
    """rps.robotarium.Robotarium without the figure or real-time pacing: poses (3, N) live on the
    GPU; get_poses / set_velocities / step follow the rps call protocol (cross_and_rescue.py:59,
    100, 170, 175)."""

    def __init__(self, number_of_robots, initial_conditions, wheel_threshold=True):
        torch = _lib.require_gpu()
        ic = np.asarray(initial_conditions, dtype=np.float64)
        if ic.shape != (3, number_of_robots):
            raise ValueError(f"initial_conditions must be (3, {number_of_robots}), got {ic.shape}")
        self.u = unicycle_params(wheel_threshold=wheel_threshold)
        self.poses = torch.tensor(np.ascontiguousarray(ic.T), device="cuda")
        self.velocities = torch.zeros((number_of_robots, 2), dtype=torch.float64, device="cuda")

    def get_poses(self):
        return self.poses.cpu().numpy().T.copy()

    def set_velocities(self, ids, velocities):
        torch = _lib.require_gpu()
        v = _dev_tensor(velocities, torch, self.poses.device, 2)
        self.velocities[torch.as_tensor(np.asarray(ids), device=self.poses.device)] = v

    def step(self):
        unicycle_advance(self.u, self.poses, self.velocities, mode=2)


class CrossAndRescue:
    """cross_and_rescue.py:29-175 as shipped, device-resident (SURVEY cfg1 with rps-lite):
    per step uni_to_si (+ goal column), cyclic pursuit of the 6 obstacles (L1, x0.05), rendezvous
    consensus of the 4 robots (L2 with the goal column), the per-robot CBF filter against the
    obstacles + static origin + robots (raw poses, Jacobi), si_barrier_cert(safety_radius=0.12),
    si_to_uni_dyn -> set_velocities -> unicycle step, obstacle Euler (T = 1/30)."""

    def __init__(self, params: FilterParams = None, safety_radius=0.12, T=1 / 30, wheel_threshold=True):
        torch = _lib.require_gpu()
        dev = torch.device("cuda")
        self.dev, self.T = dev, float(T)
        self.params = params or FilterParams()
        self.cp = self.params.c()
        self.N_robots, self.N_obs = 4, 6
        ic_r, ic_o = _cross_and_rescue_initial()
        self.u = unicycle_params(wheel_threshold=wheel_threshold)
        self.poses = torch.tensor(np.ascontiguousarray(ic_r.T), device=dev)          # (4, 3)
        self.obs_pos = torch.tensor(np.ascontiguousarray(ic_o.T), device=dev)        # (6, 2)
        self.cert = SiBarrierCert(safety_radius=safety_radius)
        th = -np.pi / self.N_obs
        self.rot = (float(np.cos(th)), float(np.sin(th)))
        self.ring = csr_from_rows([[(i + 1) % self.N_obs] for i in range(self.N_obs)], dev)   # L1, :79-86
        self.l2 = csr_from_rows([[4], [0, 3], [0, 1], [0, 2]], dev)                           # L2, :89-95
        self.goal = torch.tensor([[1.5, 0.0]], dtype=torch.float64, device=dev)               # :102
        n = self.N_obs + 1 + self.N_robots
        self.pos = torch.zeros((n, 2), dtype=torch.float64, device=dev)
        self.vel = torch.zeros((n, 2), dtype=torch.float64, device=dev)
        self.last = None

    def step(self):
        no, nr = self.N_obs, self.N_robots
        x_si = uni_to_si(self.u, self.poses)                                                  # :101
        obs_vel = consensus_csr(self.obs_pos, *self.ring, 0, None, self.rot, 0.05)            # :108-118
        si_vel = consensus_csr(x_si, *self.l2, 0, self.goal, None, 1.0)                       # :121-125
        self.pos[:no] = self.obs_pos                                                          # :130-133
        self.pos[no + 1:] = self.poses[:, :2]
        self.vel[:no] = obs_vel
        self.vel[no + 1:] = si_vel
        f = filter_swarm(self.cp, self.pos, self.vel, no + 1, method="allpairs")              # :135-160
        c = self.cert.batch(f["u"][None], x_si[None])                                         # :163
        dxu = unicycle_advance(self.u, self.poses, c["out"][0])                               # :167-175
        euler(self.obs_pos, obs_vel, self.T)                                                  # :173
        self.last = {"nominal": si_vel, "filtered": f["u"], "status": f["status"], "nbr_count": f["nbr_count"],
                     "cert": c["out"][0], "cert_status": c["status"], "x_si": x_si}
        return self.last


class MeetAtCenter:
    """meet_at_center.py:24-153 as shipped, device-resident: N unicycle robots (default 10), the
    first N/2 in cyclic pursuit on the projection points (ring, rotation -pi/(N/2)), the rest in
    complete-graph consensus (x gain; the script has gain 1); the CBF filter of every free robot
    against all obstacle robots and the other free robots (raw poses, Jacobi); si_to_uni_dyn ->
    set_velocities -> unicycle step for every robot.  The certificate is commented out in the
    script (:109) and is not applied."""

    def __init__(self, N=10, params: FilterParams = None, gain=1.0, wheel_threshold=True):
        torch = _lib.require_gpu()
        dev = torch.device("cuda")
        if N < 4 or N % 2:
            raise ValueError("N must be even and >= 4")
        self.N, self.half, self.dev = N, N // 2, dev
        self.params = params or FilterParams()
        self.cp = self.params.c()
        self.u = unicycle_params(wheel_threshold=wheel_threshold)
        self.poses = torch.tensor(np.ascontiguousarray(_meet_at_center_initial(N).T), device=dev)   # (N, 3)
        h = self.half
        th = -np.pi / h
        self.rot = (float(np.cos(th)), float(np.sin(th)))
        self.ring = csr_from_rows([[(i + 1) % h] for i in range(h)], dev)                            # L1, :65-71
        self.full = csr_from_rows([[j for j in range(h) if j != i] for i in range(h)], dev)          # completeGL, :74
        self.gain = float(gain)
        self.vel = torch.zeros((N, 2), dtype=torch.float64, device=dev)
        self.last = None

    def step(self):
        h = self.half
        x_si = uni_to_si(self.u, self.poses)                                                        # :80
        consensus_csr(x_si[:h], *self.ring, 0, None, self.rot, 1.0, out=self.vel[:h])               # :86-96
        consensus_csr(x_si[h:], *self.full, 0, None, None, self.gain, out=self.vel[h:])             # :99-103
        nominal = self.vel.clone()
        f = filter_swarm(self.cp, self.poses[:, :2].contiguous(), self.vel, h, method="allpairs")  # :114-143
        self.vel[h:] = f["u"]
        dxu = unicycle_advance(self.u, self.poses, self.vel)                                        # :148-153
        self.last = {"nominal": nominal, "filtered": self.vel.clone(), "status": f["status"],
                     "nbr_count": f["nbr_count"], "x_si": x_si}
        return self.last


def _meet_at_center_initial(N):
    """meet_at_center.py:37-48: (3, N) poses (N/2 on radius 0.7, N/2 on radius 1.05)."""
    half = N // 2
    ic = np.zeros((N, 3))
    diameter = 0.7
    for i in range(half):
        th = i * (2 * np.pi / half)
        ic[i] = np.array([0, 0, 0]) + [diameter * np.cos(th), diameter * np.sin(th), th + (2 / 3 * np.pi)]
    for i in range(half, N):
        th = i * (2 * np.pi / half) + np.pi / 5
        ic[i] = np.array([0, 0, 0]) + [1.5 * diameter * np.cos(th), 1.5 * diameter * np.sin(th),
                                       th + (2 / 3 * np.pi)]
    return ic.T.copy()


def _cross_and_rescue_initial():
    """cross_and_rescue.py:36-57: robot poses (4, 3) and obstacle positions (6, 2)."""
    N_robots, N_obs, diameter = 4, 6, 0.6
    ic_r = np.zeros((N_robots, 3))
    ic_o = np.zeros((N_obs, 2))
    for i in range(N_obs):
        th = i * (2 * np.pi / N_obs)
        ic_o[i] = np.array([0, 0]) + [diameter * np.cos(th), diameter * np.sin(th)]
    for i in range(N_robots):
        th = i * (2 * np.pi / N_robots)
        ic_r[i] = np.array([0, 0, 0]) + [0.6 * diameter * np.cos(th) - 1.15, 0.6 * diameter * np.sin(th),
                                         th + (2 / 3 * np.pi)]
    return ic_r.T.copy(), ic_o.T.copy()
