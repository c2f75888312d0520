"""Row-stripe sharding of the lattice swarm across GPUs (SURVEY 8e, cfg4 at 1/2/4/8 GPUs).

Rank r owns lattice rows [r R, (r+1) R) of a W x (R * world) lattice (weak scaling: R rows per
GPU).  One timestep depends on lattice rows up to `halo` = 4 away (cull candidates up to 3 rows
away, plus the row that forms their nominal control), so a rank that holds G = halo * k ghost rows
on each side can advance k timesteps ("sub-steps") between exchanges, recomputing the ghost rows
that are still exact.  Each exchange (every k sub-steps) is ONE collective:
  1. pack    (cbf_halo_pack_nbr)   the first G owned rows into the chunk for rank r-1, the last G
             rows into the chunk for rank r+1, and the guard records of the last k sub-steps into
             every rank's chunk;
  2. a2a     ONE all_to_all_single (RCCL over xGMI): G W 16 B of rows to each neighbour and 64 k B
             of records to every rank -- the neighbour exchange of SURVEY 8(f)1.  (exchange=
             "allgather": one all_gather_into_tensor of [first G rows | last G rows | records]
             slabs, cbf_halo_pack / cbf_halo_unpack, which delivers every rank's rows to everyone:
             (world - 1) x 2 G W 16 B per rank instead of 2 x G W 16 B.)
  3. unpack  (cbf_halo_unpack_nbr) rank r-1's last rows and rank r+1's first rows into the ghost
             rows of the window, and the halo guard of the k recorded sub-steps;
then sub-step s (cbf_lattice_step_sharded) computes rows [rb - D_s, re + D_s), D_s = G - halo (s+1)
(the owned rows at the last sub-step), over the window of those rows +- halo, with its own
workspace (so each sub-step keeps its cell order from cycle to cycle).
The guard proves that every agent outside a sub-step's candidate rows was farther than the cull
radius (in y) from every agent it computed; the records of a cycle are checked at the next
exchange, and check_guard() does one more exchange for the last ones.  Results are bit-identical
to the single-GPU step of the whole lattice whenever the guard holds (checked by tests and by
check_guard()).  The extra work is the ghost rows: about 2 G / R of the binned rows and G / R of
the computed rows per rank (k = 4, R = 1024: 3 % and 1.6 %), for a k-fold cut in collectives.

The backend object does the device work (HipBackend here; the CPU gloo tests plug in the
oracle as a backend to check the exchange logic).

Swarms that are not a lattice (GroupSwarm: cfg1/cfg2 groups, or any entity set with Laplacian
nominal controls) shard by contiguous entity ranges instead (ShardedGroupSwarm, at the end of
this module): every rank holds all positions, filters its own egos, and the new positions are
all-gathered once per timestep.
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import scenarios

RADIUS_GUARD_EPS = (1e-9, 1e-12)


def guard_ok(recs: np.ndarray, rank: int, radius: float) -> bool:
    """Host restatement of the device guard of one sub-step (k_halo_unpack): recs[q] = {min y, max
    y of q's computed rows, max y of q's owned rows below its top `guard` rows, min y above its
    bottom `guard` rows, min y, max y of q's owned rows}."""
    rm = radius * (1.0 + RADIUS_GUARD_EPS[0]) + RADIUS_GUARD_EPS[1]
    ymin, ymax = recs[rank, 0], recs[rank, 1]
    if not ymin <= ymax:
        return True
    for q in range(recs.shape[0]):
        if q < rank:
            lim = recs[q, 2] if q == rank - 1 else recs[q, 5]
            if not (ymin - lim > rm):
                return False
        elif q > rank:
            lim = recs[q, 3] if q == rank + 1 else recs[q, 4]
            if not (lim - ymax > rm):
                return False
    return True


def sub_extents(win_pos: np.ndarray, W: int, w0: int, a: int, b: int, rb: int, re: int, guard: int) -> np.ndarray:
    """The guard record of a sub-step from its input window positions (rows [w0, ...)): {min, max}
    y over computed rows [a, b), {max y of owned rows < re - guard, min y of owned rows >= rb +
    guard, min y, max y} over owned rows [rb, re)."""
    y = win_pos[:, 1].reshape(-1, W)
    comp = y[a - w0:b - w0]
    own = y[rb - w0:re - w0]
    R = own.shape[0]
    e2 = own[:R - guard].max() if R > guard else -math.inf
    e3 = own[guard:].min() if R > guard else math.inf
    return np.array([comp.min(), comp.max(), e2, e3, own.min(), own.max()], dtype=np.float64)


class Sub:
    """Geometry of sub-step s: computed rows [a, b), window [w0, w1), guard rows."""

    def __init__(self, a, b, w0, w1, guard):
        self.a, self.b, self.w0, self.w1, self.guard = a, b, w0, w1, guard


class HipBackend:
    """Device work of one rank through libcbf_amd.so."""

    def __init__(self, W, H, gain, T, params, grid, win_rows, nsub=1, nominal=None, cull="cells"):
        import torch
        from . import _lib, swarm
        self.torch, self._lib, self.swarm = torch, _lib, swarm
        # "window": every sub-step through the lattice-window cull (cbf_lattice_cycle_sharded_ex,
        # CBF_RUN_WINDOW_CULL); same results whenever the halo guard holds
        if cull not in ("cells", "window"):
            raise ValueError(f"cull must be 'cells' or 'window', got {cull!r}")
        self.cull = cull
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.W, self.H, self.gain, self.T = W, H, gain, T
        self.cp = params.c()
        self.radius = params.safety_distance
        self.grid = grid
        self.nsub = nsub
        self.ws_bytes = (_lib.lib.cbf_lattice_workspace_size(W, win_rows, _lib.C.byref(grid)) + 255) // 256 * 256
        # one workspace per sub-step (each keeps the cell order of its own window across cycles),
        # contiguous so that a whole cycle can run in one cbf_lattice_cycle_sharded call
        self.ws_all = torch.zeros((nsub * self.ws_bytes,), dtype=torch.uint8, device=self.dev)
        self.wss = [self.ws_all[s * self.ws_bytes:(s + 1) * self.ws_bytes] for s in range(nsub)]
        for w in self.wss:
            swarm.set_nominal(w, nominal)
        self.flag = torch.zeros((1,), dtype=torch.int32, device=self.dev)
        # the guard flag is read back asynchronously after every exchange: a pinned host copy per
        # exchange in flight, polled (never waited on) at the next exchanges.  The pinned words are
        # a ring allocated here, so no exchange pays a pinned allocation
        self._pending = []
        self._ring = [torch.empty((1,), dtype=torch.int32, pin_memory=True) for _ in range(8)]
        self._next = 0
        self.set_words = _lib.lib.cbf_halo_ext_bytes(1) // 8
        self.ext_keys = torch.empty((nsub * self.set_words,), dtype=torch.int64, device=self.dev)
        _lib.check(_lib.lib.cbf_halo_ext_reset(_lib.ptr(self.ext_keys), nsub, _lib.stream_handle()),
                   "cbf_halo_ext_reset")

    def tensor(self, a):
        return self.torch.as_tensor(np.ascontiguousarray(a), device=self.dev)

    # CBF_SYNC_CHECK=1 (diagnostics): synchronise after every device call, so that a device fault is
    # reported by the call that caused it (with the rank and the sub-step range) instead of by a
    # later one; the kernels' order and arguments are unchanged.
    _sync_check = __import__("os").environ.get("CBF_SYNC_CHECK", "0") == "1"

    def _checked(self, what, S):
        if self._sync_check and not self.torch.cuda.is_current_stream_capturing():
            try:
                self.torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"rank {S.rank}: device fault in {what}") from e

    def pack(self, S):
        L, P = self._lib, self._lib.ptr
        if S.exchange_mode == "neighbour":
            L.check(L.lib.cbf_halo_pack_nbr(self.W, S.G, S.n_owned, P(S.own), P(self.ext_keys), self.nsub, S.ws,
                                            S.rank, P(S.send), L.stream_handle()), "cbf_halo_pack_nbr")
            self._checked("cbf_halo_pack_nbr", S)
            return
        L.check(L.lib.cbf_halo_pack(self.W, S.G, S.n_owned, P(S.own), P(self.ext_keys), self.nsub, P(S.send),
                                    L.stream_handle()), "cbf_halo_pack")

    def unpack_guard(self, S):
        L, P = self._lib, self._lib.ptr
        if S.exchange_mode == "neighbour":
            L.check(L.lib.cbf_halo_unpack_nbr(self.W, S.G, S.rb - S.w0, S.w1 - S.re, S.re - S.w0, P(S.recv), S.ws,
                                              S.rank, self.radius, self.nsub, P(S.wpos), P(self.flag),
                                              L.stream_handle()), "cbf_halo_unpack_nbr")
            self._checked("cbf_halo_unpack_nbr", S)
            return
        L.check(L.lib.cbf_halo_unpack(self.W, S.G, S.rb - S.w0, S.w1 - S.re, S.re - S.w0, P(S.recv), S.stride,
                                      S.ws, S.rank, self.radius, self.nsub, P(S.wpos), P(self.flag),
                                      L.stream_handle()), "cbf_halo_unpack")

    def lattice_step(self, S, s, sub):
        if self.cull == "window":   # one sub-step = a cycle call of one sub-step
            self.lattice_cycle(S, s, s + 1)
            return
        L, P, W = self._lib, self._lib.ptr, self.W
        o = (sub.a - S.w0) * W
        L.check(L.lib.cbf_lattice_step_sharded(
            self.cp, L.C.byref(self.grid), W, self.H, sub.a, sub.b, S.rb, S.re, sub.w0, sub.w1 - sub.w0,
            P(S.wpos[(sub.w0 - S.w0) * W:]), self.gain, self.T, P(S.wpos[o:]), P(S.wvel[o:]), P(S.wu[o:]),
            P(S.wstatus[o:]), P(S.wcnt[o:]), sub.guard, P(self.ext_keys[s * self.set_words:]), P(S.stats_ptr()),
            P(self.wss[s]), self.ws_bytes, L.stream_handle()), "cbf_lattice_step_sharded")

    def lattice_cycle(self, S, s0=0, s1=None):
        """Sub-steps [s0, s1) of an exchange cycle, by default all nsub (cbf_lattice_cycle_sharded:
        the sub-steps after the first are binned by the previous sub-step's advance)."""
        L, P = self._lib, self._lib.ptr
        s1 = self.nsub if s1 is None else s1
        L.check(L.lib.cbf_lattice_cycle_sharded_ex(
            self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, S.halo, self.nsub, s0, s1, S.w0, S.win_rows,
            P(S.wpos), self.gain, self.T, P(S.wvel), P(S.wu), P(S.wstatus), P(S.wcnt), P(self.ext_keys),
            P(S.stats_ptr()), P(self.ws_all), self.ws_bytes, L.RUN_WINDOW_CULL if self.cull == "window" else 0,
            L.stream_handle()), "cbf_lattice_cycle_sharded_ex")
        self._checked(f"cbf_lattice_cycle_sharded (sub-steps {s0}..{s1 - 1}, stats {S.collect_stats})", S)

    def lattice_build(self, S):
        L, P = self._lib, self._lib.ptr
        sub = S.subs[-1]
        if self.cull == "window":
            L.check(L.lib.cbf_lattice_window_build_ex(
                self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, sub.w0, sub.w1 - sub.w0,
                P(S.wpos[(sub.w0 - S.w0) * self.W:]), self.gain, P(S.vel), P(self.wss[-1]), self.ws_bytes,
                L.stream_handle()), "cbf_lattice_window_build_ex")
            return
        L.check(L.lib.cbf_lattice_build(self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, sub.w0,
                                        sub.w1 - sub.w0, P(S.wpos[(sub.w0 - S.w0) * self.W:]), self.gain, P(S.vel),
                                        P(self.wss[-1]), self.ws_bytes, L.stream_handle()), "cbf_lattice_build")

    def lattice_advance(self, S, mark=None, commit=True):
        L, P = self._lib, self._lib.ptr
        sub = S.subs[-1]
        if self.cull == "window":   # new owned positions into scratch (the filter reads the window throughout)
            if getattr(self, "_own_next", None) is None:
                self._own_next = self.torch.empty_like(S.own)
            L.check(L.lib.cbf_lattice_window_advance_ex(
                self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, sub.w0, sub.w1 - sub.w0,
                P(S.wpos[(sub.w0 - S.w0) * self.W:]), self.T, P(self._own_next), P(S.u), P(S.status),
                P(S.nbr_count), P(S.stats_ptr()), P(self.wss[-1]), self.ws_bytes,
                L.C.c_void_p(mark.cuda_event if mark is not None else 0), L.stream_handle()),
                "cbf_lattice_window_advance_ex")
            if commit:
                S.own.copy_(self._own_next)
            return
        L.check(L.lib.cbf_lattice_advance_marked(
            self.cp, L.C.byref(self.grid), self.W, self.H, S.rb, S.re, sub.w0, sub.w1 - sub.w0,
            P(S.wpos[(sub.w0 - S.w0) * self.W:]), self.T, P(S.own), P(S.u), P(S.status), P(S.nbr_count), sub.guard,
            None, P(S.stats_ptr()), P(self.wss[-1]), self.ws_bytes,
            L.C.c_void_p(mark.cuda_event if mark is not None else 0), L.stream_handle()), "cbf_lattice_advance_marked")

    def arm_guard_readback(self):
        """Queue a copy of the guard flag to pinned host memory behind this exchange's unpack."""
        torch = self.torch
        while len(self._pending) >= len(self._ring) - 1:  # the oldest read-back is still in flight
            ev, host = self._pending.pop(0)
            ev.synchronize()
            if int(host[0]):
                self._failed_late = True
        host = self._ring[self._next % len(self._ring)]
        self._next += 1
        host.copy_(self.flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending.append((ev, host))

    def poll_guard(self) -> bool:
        """True once a completed exchange's guard has failed (does not wait for the GPU)."""
        if getattr(self, "_failed_late", False):
            return True
        while self._pending and self._pending[0][0].query():
            _, host = self._pending.pop(0)
            if int(host[0]):
                return True
        return False

    def guard_failed(self) -> bool:
        return bool(self.flag.item())


def ranks_share_gpu(world_size, group=None):
    """Whether two ranks of the group run on one GPU.  With torch.distributed initialised and a
    GPU visible this is decided from the real placement: every rank contributes (host, the
    device's UUID or PCI location) once, and any repeat means time-sharing (e.g. every rank of a
    rehearsal pinned to cuda:0).  Otherwise, from the counts: this node runs more ranks
    (LOCAL_WORLD_SIZE, set by torchrun and by bench.py's launcher) than it has visible GPUs."""
    import os
    import torch
    import torch.distributed as dist
    if world_size > 1 and dist.is_available() and dist.is_initialized() and torch.cuda.is_available():
        import socket
        dev = torch.cuda.current_device()
        prop = torch.cuda.get_device_properties(dev)
        where = str(getattr(prop, "uuid", "")) or \
            f"{getattr(prop, 'pci_domain_id', 0)}:{getattr(prop, 'pci_bus_id', 0)}:{getattr(prop, 'pci_device_id', dev)}"
        keys = [None] * dist.get_world_size(group)
        dist.all_gather_object(keys, (socket.gethostname(), where), group=group)
        return len(set(keys)) < len(keys)
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world_size))
    return local > max(1, torch.cuda.device_count())


class ShardedLattice:
    """One rank's stripe of a W x (rows_per_rank * world) lattice swarm (see module docstring)."""

    def __init__(self, W, rows_per_rank, seed=0, halo=4, substeps=4, gain=scenarios.LATTICE_GAIN, T=scenarios.T,
                 params=None, backend=None, group=None, pos_global=None, spacing=scenarios.LATTICE_SPACING,
                 nominal=None, exchange="neighbour", cull="cells"):
        import torch
        import torch.distributed as dist
        from .swarm import FilterParams, make_grid
        self.torch, self.dist, self.group = torch, dist, group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.W, self.R, self.halo, self.k = W, rows_per_rank, halo, substeps
        self.G = halo * substeps
        if not (2 <= halo and 1 <= substeps and self.G <= rows_per_rank):
            raise ValueError("need halo >= 2, substeps >= 1 and halo * substeps <= rows_per_rank")
        self.H = rows_per_rank * self.ws
        self.rb, self.re = self.rank * rows_per_rank, (self.rank + 1) * rows_per_rank
        self.w0 = max(0, self.rb - self.G)
        self.w1 = min(self.H, self.re + self.G)
        self.win_rows = self.w1 - self.w0
        self.subs = []
        for s in range(substeps):
            d = self.G - halo * (s + 1)
            a, b = max(0, self.rb - d), min(self.H, self.re + d)
            self.subs.append(Sub(a, b, max(0, a - halo), min(self.H, b + halo), d + halo - 1))
        # ranks time-sharing one GPU (a rehearsal on one card): the window cull's row guard from a
        # separate kernel, since a block polling for the in-launch hand-off can wait for long there
        # (cbf_params.launch_flags; results are identical)
        self.params = params or FilterParams()
        if self.params.window_guard == "auto" and ranks_share_gpu(self.ws, group):
            import dataclasses
            self.params = dataclasses.replace(self.params, window_guard="separate")
        if pos_global is None:
            pos_global = scenarios.lattice(W, self.H, seed=seed, spacing=spacing)
        win = pos_global[self.w0 * W:self.w1 * W]
        a = spacing
        grid = make_grid(-1.0 - a, self.w0 * a - 1.0 - a, W * a + 1.0, self.w1 * a + 1.0,
                         self.params.safety_distance * 1.02)
        if backend is None:
            backend = HipBackend(W, self.H, gain, T, self.params, grid, self.win_rows, substeps, nominal, cull)
        self.be = backend
        t = backend.tensor
        self.wpos = t(win)
        self.n_owned = rows_per_rank * W
        o0 = (self.rb - self.w0) * W
        self.own = self.wpos[o0:o0 + self.n_owned]
        # per-window-row outputs (sub-steps write their computed rows); the owned rows are views
        nw = self.win_rows * W
        self.wvel = t(np.zeros((nw, 2)))
        self.wu = t(np.zeros((nw, 2)))
        self.wstatus = t(np.zeros(nw, np.int32))
        self.wcnt = t(np.zeros(nw, np.int32))
        self.vel = self.wvel[o0:o0 + self.n_owned]
        self.u = self.wu[o0:o0 + self.n_owned]
        self.status = self.wstatus[o0:o0 + self.n_owned]
        self.nbr_count = self.wcnt[o0:o0 + self.n_owned]
        self.stats = t(np.zeros(1024, np.int64))  # rollout statistics, include/cbf_amd.h CBF_STAT_*
        # collect_stats=False passes stats=NULL (no statistics bookkeeping; results bit-identical)
        self.collect_stats = True
        if exchange not in ("neighbour", "allgather"):
            raise ValueError(f"exchange must be 'neighbour' or 'allgather', got {exchange!r}")
        self.exchange_mode = exchange
        self.slab = 2 * self.G * W * 2      # doubles of the first + last G owned rows
        self.stride = self.slab + 8 * substeps
        if exchange == "neighbour":
            # chunk q (to / from rank q) = [k records of 8 doubles | G rows if q = rank +- 1]
            self.splits = self.nbr_splits(self.ws, self.rank, self.G * W * 2, substeps)
            self.send = t(np.zeros(sum(self.splits)))
            self.recv = t(np.zeros(sum(self.splits)))
        else:
            # all-gather: send slab [first G rows | last G rows | k records], world slabs received
            self.send = t(np.zeros(self.stride))
            self.recv = t(np.zeros(self.stride * self.ws))
        self.use_gloo = dist.get_backend(group) == "gloo"
        # captured device work, keyed by collect_stats (the statistics pointer is baked into a graph)
        self.graphs = {}         # per-sub-step graphs (capture())
        self.cycle_graphs = {}   # whole-cycle graphs (capture_cycle())
        self.sub = 0  # next sub-step of the current exchange cycle

    @staticmethod
    def nbr_splits(ws, rank, rows_elems, nsub):
        """Chunk sizes (doubles) of the neighbour exchange's send and receive buffers, in rank
        order: every rank gets this rank's 8 nsub doubles of guard records, ranks rank - 1 and
        rank + 1 also its first / last G rows (rows_elems doubles); receiving mirrors it
        (cbf_halo_nbr_elems, nbr_chunk_off in swarm.hip)."""
        return [8 * nsub + (rows_elems if abs(q - rank) == 1 else 0) for q in range(ws)]

    def chunk_offset(self, q):
        """Offset (doubles) of chunk q in the neighbour exchange's send / receive buffer."""
        return sum(self.splits[:q])

    # ---- one timestep -------------------------------------------------------------------------
    def _collective(self):
        """The exchange's one collective: all_to_all_single of the neighbour chunks (default) or
        all_gather of the slabs.  RCCL works on the device buffers; gloo (the CPU tests, or a 1-GPU
        rehearsal of several ranks) on host copies."""
        dist = self.dist
        staged = self.use_gloo and self.send.is_cuda
        send = self.send.cpu() if staged else self.send
        recv = self.recv.cpu() if staged else self.recv
        if self.exchange_mode == "neighbour":
            dist.all_to_all_single(recv, send, self.splits, self.splits, group=self.group)
        elif self.use_gloo:
            dist.all_gather(list(recv.view(self.ws, self.stride).unbind(0)), send, group=self.group)
        else:
            dist.all_gather_into_tensor(recv, send, group=self.group)
        if staged:
            self.recv.copy_(recv)

    def exchange(self):
        # the guard of the sub-steps certified at earlier exchanges, read back without waiting:
        # a breach stops the rollout one or two cycles after it happened, not at the end
        if self.be.poll_guard():
            raise RuntimeError(self._guard_msg())
        self.be.pack(self)
        self._collective()
        self.be.unpack_guard(self)
        self.be.arm_guard_readback()

    def time_exchange(self, reps=10):
        """Wall time of this rank's exchange, split into its parts (µs per exchange, mean over reps):
        pack (device), the collective (RCCL; gloo: incl. its host staging), unpack + guard (device),
        each part closed by a device synchronize, every repetition opened by a barrier so that the
        ranks start together.  Untimed diagnostics: the state is snapshot and restored around it."""
        torch, dist = self.torch, self.dist
        snap = self.snapshot()
        parts = np.zeros(3)
        for _ in range(reps):
            dist.barrier(group=self.group)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.be.pack(self)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            self._collective()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            self.be.unpack_guard(self)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            parts += (t1 - t0, t2 - t1, t3 - t2)
        self.restore(snap)
        us = parts / reps * 1e6
        return {"pack_us": float(us[0]), "collective_us": float(us[1]), "unpack_guard_us": float(us[2]),
                "exchange_us": float(us.sum()), "exchange_us_per_timestep": float(us.sum()) / self.k,
                "timesteps_per_exchange": self.k, "bytes_sent": self.exchange_bytes()}

    def exchange_bytes(self):
        """Bytes this rank sends per exchange (rows + guard records, self excluded)."""
        if self.exchange_mode == "neighbour":
            return 8 * (sum(self.splits) - self.splits[self.rank])
        return 8 * self.stride * (self.ws - 1)

    def _guard_msg(self):
        return (f"rank {self.rank}: halo guard failed -- an agent moved within the cull radius of a stripe from "
                f"outside the {self.halo}-row halo; raise halo")

    def step(self):
        if self.sub == 0:
            self.exchange()
        graph = self.graphs.get(self.collect_stats)
        if graph is not None:
            graph[self.sub].replay()
        else:
            self.be.lattice_step(self, self.sub, self.subs[self.sub])
        self.sub = (self.sub + 1) % self.k

    def run(self, steps):
        """`steps` timesteps: the sub-steps of each exchange cycle run as one device call (a whole
        cycle, or the part of one that is left; one hipGraph replay per whole cycle after
        capture_cycle()), each after the cycle's exchange -- the same results as `steps` step()
        calls."""
        done = 0
        while done < steps:
            if not hasattr(self.be, "lattice_cycle"):
                self.step()
                done += 1
                continue
            if self.sub == 0:
                self.exchange()
            n = min(self.k - self.sub, steps - done)
            cycle_graph = self.cycle_graphs.get(self.collect_stats)
            if n == self.k and cycle_graph is not None:
                cycle_graph.replay()
            else:   # a whole cycle, or the sub-steps left of one: one call (its first sub-step bins)
                self.be.lattice_cycle(self, self.sub, self.sub + n)
            self.sub = (self.sub + n) % self.k
            done += n

    def build_phase(self):
        self.be.lattice_build(self)

    def advance_phase(self, mark=None, commit=True):
        """The last sub-step's filter + clip + Euler alone (after build_phase()), the bench's kernel
        timing.  Both culls advance the owned positions; with the window cull the new positions go
        to a scratch tensor first (its filter reads the window throughout) and commit=False leaves
        them there (the state stays, as LatticeSwarm.advance_phase(commit=False)); the cell list
        writes them in place whatever commit says."""
        self.be.lattice_advance(self, mark, commit)

    def capture(self):
        """Capture each sub-step's device work (cbf_lattice_step_sharded) into its own hipGraph,
        for the current collect_stats (graphs are kept per setting: the statistics pointer is part
        of the captured launches); the exchange (pack, collective, unpack) stays eager at the start
        of a cycle.  Capture is thread-local, so a communicator's watchdog thread is unaffected."""
        torch = self.torch
        if not self.own.is_cuda:
            return None
        torch.cuda.synchronize()
        graphs = []
        for s in range(self.k):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.be.lattice_step(self, s, self.subs[s])
            graphs.append(g)
        self.graphs[self.collect_stats] = graphs
        return graphs

    def capture_cycle(self):
        """Capture one whole exchange cycle's device work (the cbf_lattice_cycle_sharded call: k
        sub-steps, ~5 launches each) into one hipGraph, for the current collect_stats, that run()
        replays after each exchange; the exchange itself (pack, collective, unpack) stays eager.
        Capture launches nothing, so the swarm does not advance."""
        torch = self.torch
        if not self.own.is_cuda or not hasattr(self.be, "lattice_cycle"):
            return None
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.be.lattice_cycle(self)
        self.cycle_graphs[self.collect_stats] = g
        return g

    def stats_ptr(self):
        return self.stats if self.collect_stats else None

    def snapshot(self):
        """Copies of this rank's whole device state (window positions and outputs, exchange slabs,
        statistics, the backend's workspaces, guard keys and flag) and the cycle position, for
        restore().  Call after a synchronize; pending guard read-backs are settled first."""
        self.torch.cuda.synchronize()
        if self.be.poll_guard():
            raise RuntimeError(self._guard_msg())
        return (self.sub, [t.clone() for t in self._state()])

    def restore(self, snap):
        """Back to a snapshot(): the following steps repeat its trajectory bit for bit."""
        self.torch.cuda.synchronize()
        if self.be.poll_guard():
            raise RuntimeError(self._guard_msg())
        self.be._pending.clear()
        self.sub = snap[0]
        for t, c in zip(self._state(), snap[1]):
            t.copy_(c)

    def _state(self):
        ts = [self.wpos, self.wvel, self.wu, self.wstatus, self.wcnt, self.stats, self.send, self.recv]
        return ts + [self.be.ws_all, self.be.flag, self.be.ext_keys]

    def reset_solves(self):
        self.stats.zero_()

    def stats_summary(self) -> dict:
        """This rank's rollout statistics over its owned rows (include/cbf_amd.h CBF_STAT_*)."""
        from . import _lib
        st = _lib.decode_stats(self.stats.cpu().numpy())
        if st["errors"]:
            raise _lib.CbfError(f"rank {self.rank}: {st['errors']} step(s) ran on an unusable cell list")
        return st

    def solves_total(self) -> int:
        return self.stats_summary()["solves"]

    def check_guard(self):
        """Certify the sub-steps since the last exchange (one more exchange, which also refreshes
        the ghost rows) and raise if any sub-step's guard failed."""
        self.exchange()
        if self.be.guard_failed():
            raise RuntimeError(self._guard_msg())

    def owned_positions(self):
        return self.own


# ---- any swarm: contiguous entity ranges, one all-gather of the positions per timestep ----------

class HipGroupBackend:
    """Device work of ShardedGroupSwarm through the C ABI (cbf_amd.swarm)."""

    def __init__(self, groups, params, method, pos0):
        import torch
        from . import swarm
        self.torch, self.swarm = torch, swarm
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.cp = params.c()
        self.method = "allpairs" if method == "auto" and len(pos0) <= 8192 else ("cells" if method == "auto" else method)
        # the cell grid of the whole swarm, fixed at the start (with a margin; agents that drift
        # outside it fall into the edge cells, which only lengthens their candidate lists)
        self.grid = swarm.grid_for_points(pos0, params.safety_distance) if self.method == "cells" else None
        self.groups = []
        for (b, e, rows, anchors, rot, scale) in groups:
            rp, col = swarm.csr_from_rows(rows, self.dev)
            anc = None if anchors is None else torch.as_tensor(np.asarray(anchors, np.float64).reshape(-1, 2),
                                                               device=self.dev).contiguous()
            self.groups.append((b, e, rp, col, anc, rot, scale))

    def tensor(self, a):
        return self.torch.as_tensor(np.ascontiguousarray(a), device=self.dev).clone()

    def nominal(self, pos, vel):
        for (b, e, rp, col, anc, rot, scale) in self.groups:
            self.swarm.consensus_csr(pos[b:e], rp, col, 0, anc, rot, scale, out=vel[b:e])

    def filter(self, pos, vel, n_obs, eb, ee):
        out = self.swarm.filter_swarm(self.cp, pos, vel, n_obs, eb, ee, method=self.method, grid=self.grid)
        return out["u"], out["status"], out["nbr_count"]

    def euler(self, pos, u, T):
        self.swarm.euler(pos, u, T)


class ShardedGroupSwarm:
    """A swarm that is not a lattice (GroupSwarm: entity groups with graph-Laplacian nominal
    controls, cfg1/cfg2 or any random swarm), sharded the way the north star plans it: rank r owns
    the contiguous entity range [b_r, e_r) (ceil(n / world) entities each), every rank holds all
    positions, and each timestep is
      1. the nominal controls of all entities (replicated: a Laplacian row reads its neighbours'
         positions, which every rank holds; cross_and_rescue.py:108-125),
      2. the filter of this rank's egos [max(n_obs, b_r), e_r) against the whole swarm
         (filter_swarm with an ego range; cross_and_rescue.py:135-160),
      3. Euler for the rank's entities (obstacles with their nominal velocity, :173),
      4. one all-gather of every rank's new positions (RCCL all_gather_into_tensor over xGMI; gloo
         for the CPU tests).
    Each entity's step reads only the gathered state, so the rollout is bit-identical to the
    single-GPU GroupSwarm.step of the whole swarm at any world size.  The work that is replicated
    (nominal controls, and the cell list or candidate set the filter scans) is O(n); the filter
    itself, the dominant part, is split.  The lattice swarm's stripes (ShardedLattice) exchange
    only ghost rows instead."""

    def __init__(self, pos, n_obs, groups, params=None, T=1 / 30, method="auto", group=None, backend=None):
        import torch
        import torch.distributed as dist
        from .swarm import FilterParams
        self.torch, self.dist, self.group = torch, dist, group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        pos = np.asarray(pos, dtype=np.float64).reshape(-1, 2)
        self.n, self.n_obs, self.T = pos.shape[0], n_obs, T
        self.chunk = -(-self.n // self.ws)
        self.b = min(self.n, self.rank * self.chunk)
        self.e = min(self.n, self.b + self.chunk)
        self.params = params or FilterParams()
        self.be = backend if backend is not None else HipGroupBackend(groups, self.params, method, pos)
        t = self.be.tensor
        self.buf = t(np.zeros((self.ws * self.chunk, 2)))   # the gathered positions (padded ranks)
        self.buf[:self.n].copy_(torch.as_tensor(pos))
        self.pos = self.buf[:self.n]
        self.vel = t(np.zeros((self.n, 2)))
        self.send = t(np.zeros((self.chunk, 2)))
        self.u = t(np.zeros((self.e - self.b, 2)))           # this rank's applied controls
        self.status = t(np.zeros(self.e - self.b, np.int32))
        self.nbr_count = t(np.zeros(self.e - self.b, np.int32))
        self.solves = 0 if not self.buf.is_cuda else torch.zeros((), dtype=torch.int64, device=self.buf.device)
        self.use_list_gather = dist.get_backend(group) == "gloo"

    def _gather(self):
        if self.use_list_gather:
            if self.send.is_cuda:   # gloo beside a GPU (1-GPU rehearsals): staged through the host
                rc = self.buf.cpu()
                self.dist.all_gather(list(rc.view(self.ws, self.chunk, 2).unbind(0)), self.send.cpu(),
                                     group=self.group)
                self.buf.copy_(rc)
            else:
                self.dist.all_gather(list(self.buf.view(self.ws, self.chunk, 2).unbind(0)), self.send,
                                     group=self.group)
        else:
            self.dist.all_gather_into_tensor(self.buf, self.send, group=self.group)

    def step(self):
        be, b, e = self.be, self.b, self.e
        be.nominal(self.pos, self.vel)
        self.u.copy_(self.vel[b:e])              # obstacles (and idle entities) keep their nominal velocity
        eb = max(self.n_obs, b)
        ee = max(eb, e)
        if ee > eb:
            u, st, cnt = be.filter(self.pos, self.vel, self.n_obs, eb, ee)
            self.u[eb - b:].copy_(u)
            self.status[eb - b:].copy_(st)
            self.nbr_count[eb - b:].copy_(cnt)
            self.solves += (cnt > 0).sum()
        self.send[:e - b].copy_(self.pos[b:e])
        be.euler(self.send[:e - b], self.u, self.T)
        self._gather()

    def run(self, steps):
        for _ in range(steps):
            self.step()

    def solves_total(self) -> int:
        """This rank's agent-QP solves (egos with >= 1 neighbour) since construction."""
        return int(self.solves)

    def owned_positions(self):
        return self.pos[self.b:self.e]
