"""Row-stripe sharding of the lattice swarm across GPUs (SURVEY 8e, cfg4 at 1/2/4/8 GPUs).

Rank r owns lattice rows [r R, (r+1) R) of a W x (R * world) lattice (weak scaling: R rows per
GPU).  Each timestep is four device operations around ONE collective:
  1. pack    (cbf_halo_pack)   the rank's first and last `halo` owned rows + 4 y-extents of the
             owned positions that the previous step's build accumulated, into one send slab;
  2. gather  ONE all_gather_into_tensor of the slabs (RCCL over xGMI) -- 2 * halo * W * 16 B per rank;
  3. unpack  (cbf_halo_unpack) rank r-1's last rows and rank r+1's first rows into the halo rows of
             the window, and the halo guard on the gathered extents;
  4. step    (cbf_lattice_step_sharded) nominal control, cell list, filter, clip, Euler for the
             owned rows, writing them in place; its build accumulates the extents of its inputs.
The halo holds `halo` rows per side; the outermost halo row only feeds the consensus of the
next row, so candidates reach halo-1 rows beyond the stripe (guard_rows = halo - 1).  The guard
proves that every agent outside a rank's candidate rows is farther than the cull radius (in y)
from every agent it owns; it runs on the extents of step t's inputs at step t+1's exchange, and
check_guard() does one last exchange for the final step.  Results are bit-identical to the
single-GPU step of the whole lattice whenever the guard holds (checked by tests and by
check_guard()).  With capture(), steps 1 and 3-4 replay as two hipGraphs around the eager
collective.

The backend object does the device work (HipBackend here; the CPU gloo tests plug in the
oracle as a backend to check the exchange logic).
"""
from __future__ import annotations

import math

import numpy as np

from . import scenarios

RADIUS_GUARD_EPS = (1e-9, 1e-12)


def guard_ok(ext_all: np.ndarray, rank: int, radius: float) -> bool:
    """Host restatement of the device guard (cbf_halo_guard)."""
    rm = radius * (1.0 + RADIUS_GUARD_EPS[0]) + RADIUS_GUARD_EPS[1]
    ymin, ymax = ext_all[rank, 0], ext_all[rank, 1]
    for q in range(ext_all.shape[0]):
        if q < rank:
            lim = ext_all[q, 2] if q == rank - 1 else ext_all[q, 1]
            if not (ymin - lim > rm):
                return False
        elif q > rank:
            lim = ext_all[q, 3] if q == rank + 1 else ext_all[q, 0]
            if not (lim - ymax > rm):
                return False
    return True


def stripe_extents(pos_rows: np.ndarray, W: int, guard_rows: int) -> np.ndarray:
    """{min y, max y, max y of rows < R - guard_rows, min y of rows >= guard_rows} of an owned stripe."""
    y = pos_rows[:, 1].reshape(-1, W)
    R = y.shape[0]
    e2 = y[:R - guard_rows].max() if R > guard_rows else -math.inf
    e3 = y[guard_rows:].min() if R > guard_rows else math.inf
    return np.array([y.min(), y.max(), e2, e3], dtype=np.float64)


class HipBackend:
    """Device work of one rank through libcbf_amd.so."""

    def __init__(self, W, H, gain, T, params, grid, win_rows):
        import torch
        from . import _lib, swarm
        self.torch, self._lib, self.swarm = torch, _lib, swarm
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.W, self.H, self.gain, self.T = W, H, gain, T
        self.cp = params.c()
        self.radius = params.safety_distance
        self.grid = grid
        self.ws_bytes = _lib.lib.cbf_lattice_workspace_size(W, win_rows, _lib.C.byref(grid))
        self.ws = torch.zeros((self.ws_bytes,), dtype=torch.uint8, device=self.dev)
        self.flag = torch.zeros((1,), dtype=torch.int32, device=self.dev)
        self.ext_keys = torch.empty((_lib.lib.cbf_halo_ext_bytes() // 8,), dtype=torch.int64, device=self.dev)
        _lib.check(_lib.lib.cbf_halo_ext_reset(_lib.ptr(self.ext_keys), _lib.stream_handle()), "cbf_halo_ext_reset")

    def tensor(self, a):
        return self.torch.as_tensor(np.ascontiguousarray(a), device=self.dev)

    def pack(self, S):
        L, P = self._lib, self._lib.ptr
        L.check(L.lib.cbf_halo_pack(self.W, S.halo, S.n_owned, P(S.own), P(self.ext_keys), P(S.send),
                                    L.stream_handle()), "cbf_halo_pack")

    def unpack_guard(self, S):
        L, P = self._lib, self._lib.ptr
        L.check(L.lib.cbf_halo_unpack(self.W, S.halo, S.rb - S.w0, S.w1 - S.re, S.re - S.w0, P(S.recv), S.stride,
                                      S.ws, S.rank, self.radius, P(S.wpos), P(self.flag), L.stream_handle()),
                "cbf_halo_unpack")

    def lattice_step(self, S):
        L, P = self._lib, self._lib.ptr
        L.check(L.lib.cbf_lattice_step_sharded(self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, S.w0,
                                               S.win_rows, P(S.wpos), self.gain, self.T, P(S.own), P(S.vel), P(S.u),
                                               P(S.status), P(S.nbr_count), S.halo - 1, P(self.ext_keys),
                                               P(S.solves), P(self.ws), self.ws_bytes, L.stream_handle()),
                "cbf_lattice_step_sharded")

    def lattice_build(self, S):
        L, P = self._lib, self._lib.ptr
        L.check(L.lib.cbf_lattice_build(self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, S.w0, S.win_rows,
                                        P(S.wpos), self.gain, P(S.vel), P(self.ws), self.ws_bytes,
                                        L.stream_handle()), "cbf_lattice_build")

    def lattice_advance(self, S):
        L, P = self._lib, self._lib.ptr
        L.check(L.lib.cbf_lattice_advance(self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, S.w0,
                                          S.win_rows, P(S.wpos), self.T, P(S.own), P(S.u), P(S.status),
                                          P(S.nbr_count), S.halo - 1, None, P(S.solves), P(self.ws),
                                          self.ws_bytes, L.stream_handle()), "cbf_lattice_advance")

    def guard_failed(self) -> bool:
        return bool(self.flag.item())


class ShardedLattice:
    """One rank's stripe of a W x (rows_per_rank * world) lattice swarm (see module docstring)."""

    def __init__(self, W, rows_per_rank, seed=0, halo=4, gain=scenarios.LATTICE_GAIN, T=scenarios.T, params=None,
                 backend=None, group=None, pos_global=None):
        import torch
        import torch.distributed as dist
        from .swarm import FilterParams, make_grid
        self.torch, self.dist, self.group = torch, dist, group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.W, self.R, self.halo = W, rows_per_rank, halo
        if not (2 <= halo <= rows_per_rank):
            raise ValueError("need 2 <= halo <= rows_per_rank")
        self.H = rows_per_rank * self.ws
        self.rb, self.re = self.rank * rows_per_rank, (self.rank + 1) * rows_per_rank
        self.w0 = max(0, self.rb - halo)
        self.w1 = min(self.H, self.re + halo)
        self.win_rows = self.w1 - self.w0
        self.params = params or FilterParams()
        if pos_global is None:
            pos_global = scenarios.lattice(W, self.H, seed=seed)
        win = pos_global[self.w0 * W:self.w1 * W]
        a = scenarios.LATTICE_SPACING
        grid = make_grid(-1.0 - a, self.w0 * a - 1.0 - a, W * a + 1.0, self.w1 * a + 1.0,
                         self.params.safety_distance * 1.02)
        if backend is None:
            backend = HipBackend(W, self.H, gain, T, self.params, grid, self.win_rows)
        self.be = backend
        t = backend.tensor
        self.wpos = t(win)
        self.n_owned = rows_per_rank * W
        o0 = (self.rb - self.w0) * W
        self.own = self.wpos[o0:o0 + self.n_owned]
        self.vel = t(np.zeros((self.n_owned, 2)))
        self.u = t(np.zeros((self.n_owned, 2)))
        self.status = t(np.zeros(self.n_owned, np.int32))
        self.nbr_count = t(np.zeros(self.n_owned, np.int32))
        self.solves = t(np.zeros(1024, np.int64))
        # send slab: [first halo rows | last halo rows | 4 extents (+4 pad)] doubles
        self.slab = 2 * halo * W * 2
        self.stride = self.slab + 8
        self.send = t(np.zeros(self.stride))
        self.recv = t(np.zeros(self.stride * self.ws))
        self.use_list_gather = dist.get_backend(group) == "gloo"
        self.graph = None

    # ---- one timestep -------------------------------------------------------------------------
    def _gather(self):
        if self.use_list_gather:   # gloo (CPU tests, or a 1-GPU rehearsal of several ranks via host staging)
            if self.send.is_cuda:
                rc = self.recv.cpu()
                self.dist.all_gather(list(rc.view(self.ws, self.stride).unbind(0)), self.send.cpu(),
                                     group=self.group)
                self.recv.copy_(rc)
            else:
                self.dist.all_gather(list(self.recv.view(self.ws, self.stride).unbind(0)), self.send,
                                     group=self.group)
        else:                      # RCCL: one all-gather into the contiguous receive slab
            self.dist.all_gather_into_tensor(self.recv, self.send, group=self.group)

    def exchange(self):
        self.be.pack(self)
        self._gather()
        self.be.unpack_guard(self)

    def _post(self):
        self.be.unpack_guard(self)
        self.be.lattice_step(self)

    def step(self):
        if self.graph is not None:   # two captured graphs around the (eager) collective
            self.graph[0].replay()
            self._gather()
            self.graph[1].replay()
            return
        self.exchange()
        self.be.lattice_step(self)

    def build_phase(self):
        self.be.lattice_build(self)

    def advance_phase(self):
        self.be.lattice_advance(self)

    def capture(self):
        """Capture the device work of a step into two hipGraphs -- the halo pack, and unpack +
        guard + the fused lattice step -- so one step is two graph launches around the eager
        collective (RCCL stays outside the graphs)."""
        torch = self.torch
        if not self.own.is_cuda:
            return None
        torch.cuda.synchronize()
        g0, g1 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g0):
            self.be.pack(self)
        with torch.cuda.graph(g1):
            self._post()
        self.graph = (g0, g1)
        return self.graph

    def reset_solves(self):
        self.solves.zero_()

    def solves_total(self) -> int:
        return int(self.solves.view(64, 16)[:, 0].sum().item())

    def check_guard(self):
        """Certify the last step (one more exchange of extents) and raise if any step's guard failed."""
        self.exchange()
        if self.be.guard_failed():
            raise RuntimeError(f"rank {self.rank}: halo guard failed -- an agent moved within the cull radius of "
                               f"a stripe from outside the {self.halo}-row halo; raise halo")

    def owned_positions(self):
        return self.own
