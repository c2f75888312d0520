"""Batched swarm API over the HIP library: the per-agent loop of the reference callers
(cross_and_rescue.py:97-175, meet_at_center.py:76-153) as device-resident batched steps.

Entity layout: one (n, 2) float64 CUDA tensor of positions and one of velocities; entities
[0, n_obs) are obstacles, [n_obs, n) agents.  An agent's "velocity" slot is its nominal control
u0 (cross_and_rescue.py:133) -- exactly the reference's packing, kept as SoA-of-pairs so every
lane loads 16 contiguous bytes.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import CbfDiag, CbfGrid, check, lib, ptr, stream_handle


@dataclass
class FilterParams:
    """ControlBarrierFunction(max_speed, dmin, k) + the callers' f, g and cull radius."""
    max_speed: float = 15.0              # cross_and_rescue.py:30
    dmin: float = 0.2                    # cbf.py:6
    k: float = 1.0                       # cbf.py:6
    safety_distance: float = 0.2         # cross_and_rescue.py:134
    f: np.ndarray = field(default_factory=lambda: np.zeros((4, 4)))                                  # :31
    g: np.ndarray = field(default_factory=lambda: 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]]))  # :32
    # lattice steps only: where the QPs that neither the origin nor one projection settles are solved
    # (cbf_params.solve_inline_max): "auto" (inline in the filter for windows of <= 131072 agents,
    # queued for the second kernel above), "inline" (always in the filter), "queued" (always the
    # queue kernel), or an int threshold.  Results are bit-identical; only the speed differs.
    solve_placement: object = "auto"
    # window cull only: where its row guard is formed (cbf_params.launch_flags): "in_filter" (the
    # filter launch's first block hands it to the others: the faster form on a GPU one process
    # owns), "separate" (a one-block kernel after the build: for ranks time-sharing one GPU), or
    # "auto" (in_filter; ShardedLattice takes separate when its node runs more ranks than GPUs).
    # Results are identical.
    window_guard: str = "auto"

    def c(self):
        p = _lib.make_params(self.max_speed, self.dmin, self.k, self.f, self.g, self.safety_distance)
        p.solve_inline_max = solve_inline_max(self.solve_placement)
        if self.window_guard not in ("auto", "in_filter", "separate"):
            raise ValueError(f"window_guard must be 'auto', 'in_filter' or 'separate', got {self.window_guard!r}")
        p.launch_flags = _lib.LAUNCH_SEPARATE_GUARD if self.window_guard == "separate" else 0
        return p


def solve_inline_max(placement) -> int:
    """cbf_params.solve_inline_max for a FilterParams.solve_placement value."""
    if isinstance(placement, (int, np.integer)) and not isinstance(placement, bool):
        if not 0 <= int(placement) < 2 ** 31:
            raise ValueError(f"solve_placement threshold out of range: {placement}")
        return int(placement)
    table = {"auto": -1, "inline": 2 ** 31 - 1, "queued": 0}
    if placement not in table:
        raise ValueError(f"solve_placement must be 'auto', 'inline', 'queued' or an int, got {placement!r}")
    return table[placement]


def make_grid(xmin, ymin, xmax, ymax, cell):
    g = CbfGrid()
    g.x0, g.y0, g.inv_h = float(xmin), float(ymin), 1.0 / float(cell)
    g.nx = max(1, int(math.ceil((xmax - xmin) / cell)))
    g.ny = max(1, int(math.ceil((ymax - ymin) / cell)))
    return g


def grid_for_points(pos_np, cull_radius, margin=1.0, cell_factor=1.02):
    """A grid over the finite points (+ margin); agents outside it are clamped into the edge cells,
    and non-finite ones never pass the cull test anyway."""
    fin = pos_np[np.isfinite(pos_np).all(axis=1)]
    if fin.shape[0] == 0:
        fin = np.zeros((1, 2))
    lo = fin.min(axis=0) - margin
    hi = fin.max(axis=0) + margin
    return make_grid(lo[0], lo[1], hi[0], hi[1], cull_radius * cell_factor)


def filter_swarm_hocbf(params, pos, vel, n_obs, ego_begin=None, ego_end=None, alpha=(1.0, 1.0), kmax=32,
                       return_x=False):
    """The swarm loop (cross_and_rescue.py:135-160 shape) with Euclidean HOCBF rows: all-pairs
    cull in reference order (cbf_cull_allpairs), then the HOCBF QP per ego
    (cbf_filter_indexed_hocbf).  kmax grows to the largest neighbour count if needed."""
    torch = _lib.require_gpu()
    n = pos.shape[0]
    eb = n_obs if ego_begin is None else ego_begin
    ee = n if ego_end is None else ego_end
    ne = ee - eb
    if not (0 <= n_obs <= eb <= ee <= n):
        raise _lib.CbfError(f"filter_swarm_hocbf: need 0 <= n_obs <= ego_begin <= ego_end <= n, got "
                            f"{n_obs}, {eb}, {ee}, {n}")
    dev = pos.device
    pos = pos.contiguous()
    vel = vel.contiguous()
    cp = params.c() if isinstance(params, FilterParams) else params
    cnt = torch.empty((ne,), dtype=torch.int32, device=dev)
    while True:
        idx = torch.empty((ne, max(kmax, 1)), dtype=torch.int32, device=dev)
        check(lib.cbf_cull_allpairs(cp, n, n_obs, ptr(pos), eb, ee, kmax, ptr(idx), ptr(cnt), stream_handle()),
              "cbf_cull_allpairs")
        need_k = int(cnt.max().item()) if ne else 0
        if need_k <= kmax:
            break
        kmax = need_k
    out = {"u": torch.empty((ne, 2), dtype=torch.float64, device=dev),
           "status": torch.empty((ne,), dtype=torch.int32, device=dev), "nbr_count": cnt, "nbr_idx": idx}
    if return_x:
        out["x"] = torch.empty((ne, 2), dtype=torch.float64, device=dev)
    need = lib.cbf_hocbf_workspace_size(ne * kmax)
    ws = torch.empty((need,), dtype=torch.uint8, device=dev)
    hp = _lib.CbfHocbf(float(alpha[0]), float(alpha[1]))
    check(lib.cbf_filter_indexed_hocbf(cp, _lib.C.byref(hp), n, ptr(pos), ptr(vel), eb, ee, kmax, ptr(idx), ptr(cnt),
                                       ptr(out["u"]), ptr(out["status"]), ptr(out.get("x")), ptr(ws), need,
                                       stream_handle()), "cbf_filter_indexed_hocbf")
    return out


def filter_swarm(params, pos, vel, n_obs, ego_begin=None, ego_end=None, method="auto", grid=None, kmax=0,
                 diag=False, workspace=None):
    """cross_and_rescue.py:135-160 for every ego in [ego_begin, ego_end).  Returns a dict of
    CUDA tensors: u (n_ego,2), status, nbr_count [, nbr_idx, nbr_active, box_active, x, viol].
    workspace (method "cells"): a zero-filled uint8 tensor bound to one (n, grid) shape on first
    use (include/cbf_amd.h); pass the same grid with it, or leave it None for a fresh one."""
    torch = _lib.require_gpu()
    n = pos.shape[0]
    eb = n_obs if ego_begin is None else ego_begin
    ee = n if ego_end is None else ego_end
    ne = ee - eb
    if not (0 <= n_obs <= eb <= ee <= n):
        raise _lib.CbfError(f"filter_swarm: need 0 <= n_obs <= ego_begin <= ego_end <= n, got "
                            f"{n_obs}, {eb}, {ee}, {n}")
    dev = pos.device
    pos = pos.contiguous()
    vel = vel.contiguous()
    assert pos.dtype == torch.float64 and vel.dtype == torch.float64 and pos.shape == vel.shape == (n, 2)
    cp = params.c() if isinstance(params, FilterParams) else params
    out = {"u": torch.empty((ne, 2), dtype=torch.float64, device=dev),
           "status": torch.empty((ne,), dtype=torch.int32, device=dev),
           "nbr_count": torch.empty((ne,), dtype=torch.int32, device=dev)}
    D = None
    if kmax or diag:
        D = CbfDiag()
        D.kmax = kmax
        if kmax:
            out["nbr_idx"] = torch.empty((ne, kmax), dtype=torch.int32, device=dev)
            D.nbr_idx = out["nbr_idx"].data_ptr()
            if diag:
                out["nbr_active"] = torch.empty((ne, kmax), dtype=torch.uint8, device=dev)
                D.nbr_active = out["nbr_active"].data_ptr()
        if diag:
            out["box_active"] = torch.empty((ne,), dtype=torch.uint8, device=dev)
            out["x"] = torch.empty((ne, 2), dtype=torch.float64, device=dev)
            out["viol"] = torch.empty((ne,), dtype=torch.float64, device=dev)
            D.box_active = out["box_active"].data_ptr()
            D.x = out["x"].data_ptr()
            D.viol = out["viol"].data_ptr()
    if method == "auto":
        method = "allpairs" if n <= 8192 else "cells"
    Dp = None if D is None else _lib.C.byref(D)
    if method == "allpairs" and D is None:
        need = lib.cbf_allpairs_workspace_size(n, ne)
        if workspace is None or workspace.numel() < need:
            workspace = torch.empty((need,), dtype=torch.uint8, device=dev)
        check(lib.cbf_filter_allpairs_split(cp, n, n_obs, ptr(pos), ptr(vel), eb, ee, ptr(out["u"]),
                                            ptr(out["status"]), ptr(out["nbr_count"]), ptr(workspace), need,
                                            stream_handle()), "cbf_filter_allpairs_split")
    elif method == "allpairs":
        check(lib.cbf_filter_allpairs(cp, n, n_obs, ptr(pos), ptr(vel), eb, ee, ptr(out["u"]), ptr(out["status"]),
                                      ptr(out["nbr_count"]), Dp, stream_handle()), "cbf_filter_allpairs")
    elif method == "cells":
        if grid is None:
            grid = grid_for_points(pos.cpu().numpy(), params.safety_distance if isinstance(params, FilterParams)
                                   else math.sqrt(cp.cull_t))
        need = lib.cbf_cells_workspace_size(n, _lib.C.byref(grid))
        if workspace is None or workspace.numel() < need:
            workspace = torch.zeros((need,), dtype=torch.uint8, device=dev)
        check(lib.cbf_filter_cells(cp, _lib.C.byref(grid), n, n_obs, ptr(pos), ptr(vel), eb, ee, ptr(out["u"]),
                                   ptr(out["status"]), ptr(out["nbr_count"]), Dp, ptr(workspace), need,
                                   stream_handle()), "cbf_filter_cells")
    else:
        raise ValueError(method)
    return out


def consensus_csr(src, row_ptr, col, self_offset=0, anchors=None, rot=None, scale=1.0, out=None):
    """Laplacian nominal control (cross_and_rescue.py:108-125): out[k] = (sum_j (x_j - x_k)) [@ R] * scale."""
    torch = _lib.require_gpu()
    n_dst = row_ptr.shape[0] - 1
    if out is None:
        out = torch.empty((n_dst, 2), dtype=torch.float64, device=src.device)
    rc, rs = (1.0, 0.0) if rot is None else rot
    check(lib.cbf_consensus_csr(n_dst, self_offset, src.shape[0], ptr(src), ptr(anchors), ptr(row_ptr), ptr(col),
                                0 if rot is None else 1, float(rc), float(rs), float(scale), ptr(out),
                                stream_handle()), "cbf_consensus_csr")
    return out


def consensus_lattice(pos, W, H, gain, row_begin=0, row_end=None, pos_row0=0, out=None):
    torch = _lib.require_gpu()
    row_end = H if row_end is None else row_end
    if out is None:
        out = torch.empty(((row_end - row_begin) * W, 2), dtype=torch.float64, device=pos.device)
    check(lib.cbf_consensus_lattice(W, H, row_begin, row_end, pos_row0, ptr(pos), float(gain), ptr(out),
                                    stream_handle()), "cbf_consensus_lattice")
    return out


def euler(pos, vel, T):
    """In place: pos <- pos + T*vel (cross_and_rescue.py:173)."""
    _lib.require_gpu()
    check(lib.cbf_euler(pos.shape[0], ptr(pos), ptr(vel), float(T), stream_handle()), "cbf_euler")
    return pos


def csr_from_rows(rows, device):
    import torch
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    col = np.array([j for r in rows for j in r] or [0], dtype=np.int32)
    return torch.tensor(rp, device=device), torch.tensor(col, device=device)


class GroupSwarm:
    """A swarm of entity groups with graph-Laplacian nominal controls (cfg1/cfg2 shape):
    each group = (begin, end, rows [list of neighbour lists, indices relative to begin;
    >= size -> anchors], anchors, rotation (c, s) or None, scale).  One step = nominal control
    per group, per-agent cull + filter (all-pairs) for egos [n_obs, n), Euler for every entity
    (obstacles with their nominal velocity, agents with the filtered control)."""

    def __init__(self, pos, n_obs, groups, params: FilterParams = None, T=1 / 30, method="auto"):
        torch = _lib.require_gpu()
        self.dev = torch.device("cuda")
        self.pos = torch.as_tensor(np.asarray(pos, dtype=np.float64), device=self.dev).contiguous()
        self.n = self.pos.shape[0]
        self.n_obs = n_obs
        self.T = T
        self.params = params or FilterParams()
        self.cp = self.params.c()
        self.method = method
        self.vel = torch.zeros_like(self.pos)
        self.groups = []
        for (b, e, rows, anchors, rot, scale) in groups:
            rp, col = csr_from_rows(rows, self.dev)
            anc = None if anchors is None else torch.as_tensor(np.asarray(anchors, np.float64).reshape(-1, 2),
                                                               device=self.dev).contiguous()
            self.groups.append((b, e, rp, col, anc, rot, scale))
        self.last = None

    def nominal(self):
        for (b, e, rp, col, anc, rot, scale) in self.groups:
            consensus_csr(self.pos[b:e], rp, col, 0, anc, rot, scale, out=self.vel[b:e])
        return self.vel

    def step(self, kmax=0, diag=False):
        self.nominal()
        out = filter_swarm(self.cp, self.pos, self.vel, self.n_obs, method=self.method, kmax=kmax, diag=diag)
        u = self.vel.clone()
        u[self.n_obs:] = out["u"]
        out["nominal"] = self.vel.clone()
        out["u_all"] = u
        euler(self.pos, u, self.T)
        self.last = out
        return out


def set_nominal(ws, nominal):
    """Bind a lattice workspace's nominal control (cbf_lattice_set_nominal): None or "consensus",
    or ("random", amp, seed).  Returns the normalised spec."""
    if nominal is None or nominal == "consensus":
        return None
    kind, amp, seed = nominal
    if kind != "random":
        raise ValueError(f"nominal must be 'consensus' or ('random', amp, seed), got {nominal!r}")
    check(lib.cbf_lattice_set_nominal(ptr(ws), ws.numel(), 1, float(amp), int(seed) & (2 ** 64 - 1),
                                      stream_handle()), "cbf_lattice_set_nominal")
    return ("random", float(amp), int(seed))


class LatticeSwarm:
    """SURVEY cfg3/cfg4: a W x H lattice swarm, one fused timestep per `step()` through
    cbf_lattice_step (nominal + cell list + filter + clip + Euler); optionally captured in a
    hipGraph.  Single-GPU: the window is the whole lattice."""

    # cull="auto": the share of egos per timestep that took the window cull's unbounded walk above
    # which the swarm switches to the cell list, and how many timesteps pass between looks
    AUTO_WALK_FRACTION = 0.01
    AUTO_CHECK_STEPS = 8

    def __init__(self, pos, W, H, gain=0.25, params: FilterParams = None, T=1 / 30, grid=None, margin=1.0,
                 method="cells", barrier="reference", alpha=(1.0, 1.0), nominal=None, cull="cells"):
        torch = _lib.require_gpu()
        # cull (reference barrier, cell method): "cells" = the cell-list cull rebuilt every timestep;
        # "window" = the lattice-window cull (include/cbf_amd.h CBF_RUN_WINDOW_CULL: candidates are the
        # lattice neighbours, guards prove the rest out of range; bit-identical results, no cell-list
        # build -- fast while the swarm stays lattice-like, e.g. under consensus); "auto" = the window
        # cull while it stays on its fast path, the cell list (for the rest of the rollout) once more
        # than AUTO_WALK_FRACTION of the egos per timestep had to walk (cbf_lattice_window_counters,
        # read without blocking every AUTO_CHECK_STEPS timesteps).  Results are identical whichever runs.
        if cull not in ("cells", "window", "auto"):
            raise ValueError(f"cull must be 'cells', 'window' or 'auto', got {cull!r}")
        window_ok = method == "cells" and barrier == "reference" and 4 <= W <= 2048
        if cull == "window" and not window_ok:
            raise ValueError("the window cull needs the reference barrier, method='cells' and 4 <= W <= 2048")
        self.cull_mode = cull
        self.cull = "window" if cull == "window" or (cull == "auto" and window_ok) else "cells"
        self._auto = None if cull != "auto" or self.cull != "window" else \
            {"steps": 0, "base": (0, 0), "pending": None, "host": torch.zeros(2, dtype=torch.int64, pin_memory=True)}
        self.dev = torch.device("cuda")
        pos = np.asarray(pos, dtype=np.float64).reshape(W * H, 2)
        self.W, self.H, self.gain, self.T = W, H, float(gain), float(T)
        self.method = method  # "cells" (fused cbf_lattice_step) or "allpairs" (cfg3: every pair tested)
        if barrier not in ("reference", "euclidean_hocbf"):
            raise ValueError(f"barrier must be 'reference' or 'euclidean_hocbf', got {barrier!r}")
        if barrier != "reference" and method != "cells":
            raise ValueError("the Euclidean HOCBF lattice step uses the cell list (method='cells')")
        self.barrier = barrier
        self.alpha = (float(alpha[0]), float(alpha[1]))
        self.hp = _lib.CbfHocbf(float(alpha[0]), float(alpha[1]))
        self.params = params or FilterParams()
        self.cp = self.params.c()
        self.grid = grid or grid_for_points(pos, self.params.safety_distance, margin=margin)
        n = W * H
        self.n = n
        self.pos = torch.tensor(pos, device=self.dev)
        self.vel = torch.empty((n, 2), dtype=torch.float64, device=self.dev)
        self.u = torch.empty((n, 2), dtype=torch.float64, device=self.dev)
        self.status = torch.empty((n,), dtype=torch.int32, device=self.dev)
        self.nbr_count = torch.empty((n,), dtype=torch.int32, device=self.dev)
        self.ws_bytes = lib.cbf_lattice_workspace_size(W, H, _lib.C.byref(self.grid))
        self.ws = torch.zeros((self.ws_bytes,), dtype=torch.uint8, device=self.dev)
        # nominal control: None / "consensus" = the lattice Laplacian (gain); ("random", amp, seed)
        # = the synthetic random walk of include/cbf_amd.h CBF_NOMINAL_RANDOM (cell method only)
        if nominal not in (None, "consensus") and method != "cells":
            raise ValueError("a random-walk nominal control needs the cell method (the lattice builds form it)")
        self.nominal = set_nominal(self.ws, nominal)
        # rollout statistics of the fused step (include/cbf_amd.h CBF_STAT_*: solves, status counts,
        # violations, minimum neighbour distance), accumulated on device by every step
        self.stats = torch.zeros((1024,), dtype=torch.int64, device=self.dev)
        # collect_stats=False passes stats=NULL: the kernels skip the statistics bookkeeping (the
        # reference computes none of it); results are bit-identical either way
        self.collect_stats = True
        self.ap_ws = torch.empty((lib.cbf_allpairs_workspace_size(n, n) if method == "allpairs" else 1,),
                                 dtype=torch.uint8, device=self.dev)
        self.graphs = {}      # captured step() graphs, keyed by collect_stats
        self.run_graphs = {}  # captured run(steps) graphs, keyed by (steps, collect_stats, history)
        self._hist = {}       # per-timestep output arrays of run(steps, history=True), keyed by steps

    def _st(self):
        return ptr(self.stats) if self.collect_stats else None

    def _launch(self):
        if self.method == "allpairs":
            consensus_lattice(self.pos, self.W, self.H, self.gain, out=self.vel)
            check(lib.cbf_filter_allpairs_split(self.cp, self.n, 0, ptr(self.pos), ptr(self.vel), 0, self.n,
                                                ptr(self.u), ptr(self.status), ptr(self.nbr_count),
                                                ptr(self.ap_ws), self.ap_ws.numel(), stream_handle()),
                  "cbf_filter_allpairs_split")
            euler(self.pos, self.u, self.T)
            if self.collect_stats:
                self.stats[_lib.STAT_SOLVES] += (self.nbr_count > 0).sum()
            return
        if self.barrier == "euclidean_hocbf":
            self.build_phase()
            self.advance_phase()
            return
        if self.cull == "window":  # one window-cull timestep (pos advanced in place through the workspace)
            self._launch_run(1)
            return
        check(lib.cbf_lattice_step(self.cp, _lib.C.byref(self.grid), self.W, self.H, 0, self.H, 0, self.H,
                                   ptr(self.pos), self.gain, self.T, ptr(self.pos), ptr(self.vel), ptr(self.u),
                                   ptr(self.status), ptr(self.nbr_count), 0, None, self._st(), ptr(self.ws),
                                   self.ws_bytes, stream_handle()), "cbf_lattice_step")

    def _history(self, steps):
        """Per-timestep output arrays for run(steps, history=True): (vel, u, status, nbr_count) of
        `steps` timesteps, grown as needed (the graphs of a size keep their buffers)."""
        import torch
        h = self._hist.get(steps)
        if h is None:
            n, dev = self.n, self.dev
            h = (torch.empty((steps, n, 2), dtype=torch.float64, device=dev),
                 torch.empty((steps, n, 2), dtype=torch.float64, device=dev),
                 torch.empty((steps, n), dtype=torch.int32, device=dev),
                 torch.empty((steps, n), dtype=torch.int32, device=dev))
            self._hist[steps] = h
        return h

    def _launch_run(self, steps, history=False):
        if self.barrier == "euclidean_hocbf":  # no fused multi-step launch: `steps` single timesteps
            if history:
                raise ValueError("run(history=True) is the reference barrier's (cbf_lattice_run_ex)")
            for _ in range(steps):
                self._launch()
            return
        if history:
            vel, u, st, cnt = self._history(steps)
            flags = _lib.RUN_OUTPUT_HISTORY
        else:
            vel, u, st, cnt, flags = self.vel, self.u, self.status, self.nbr_count, 0
        if self.cull == "window":
            flags |= _lib.RUN_WINDOW_CULL
        check(lib.cbf_lattice_run_ex(self.cp, _lib.C.byref(self.grid), self.W, self.H, ptr(self.pos), self.gain,
                                     self.T, steps, ptr(vel), ptr(u), ptr(st), ptr(cnt), self._st(), ptr(self.ws),
                                     self.ws_bytes, flags, stream_handle()), "cbf_lattice_run_ex")

    def run(self, steps, history=False):
        """`steps` timesteps through cbf_lattice_run (bit-identical to `steps` step() calls; the
        bin pass runs once, later timesteps are binned by the previous advance).  Reference
        barrier, cell method.  history=True stores every timestep's nominal control, filtered
        control, status and neighbour count (the reference's per-step si_velocities,
        cross_and_rescue.py:159-160) in the arrays of history(steps) instead of the last one only.
        The Euclidean HOCBF barrier (cell method, no history): `steps` step() launches, replayed as
        one hipGraph once capture(steps) has recorded them (no per-timestep graph launch)."""
        if self.method != "cells":
            raise ValueError("run() is the multi-step path of the cell method")
        g = self.run_graphs.get((steps, self.collect_stats, history, self.cull))
        if g is not None:
            g.replay()
        else:
            self._launch_run(steps, history)
        self._auto_check(steps)

    def window_counters(self):
        """(egos that took the window cull's unbounded walk, row-guard words read at their spin limit)
        accumulated in this swarm's workspace (cbf_lattice_window_counters; synchronises the stream).
        Both stay 0 under the cell list."""
        torch = _lib.require_gpu()
        out = torch.zeros(2, dtype=torch.int64, pin_memory=True)
        check(lib.cbf_lattice_window_counters(ptr(self.ws), self.ws_bytes, ptr(out), stream_handle()),
              "cbf_lattice_window_counters")
        torch.cuda.current_stream().synchronize()
        return int(out[0]), int(out[1])

    def _auto_check(self, steps):
        """cull="auto": every AUTO_CHECK_STEPS timesteps queue a copy of the window counters behind the
        work (pinned host memory, an event); once a copy has landed (polled, never waited for), switch
        to the cell list if the walks per ego and timestep since the previous look exceed
        AUTO_WALK_FRACTION."""
        A = self._auto
        if A is None or self.cull != "window":
            return
        A["steps"] += steps
        pend = A["pending"]
        if pend is not None and pend[0].query():
            walks, stalls = int(A["host"][0]), int(A["host"][1])
            base = A["base"]
            A["base"], A["pending"] = (walks, stalls), None
            if base is None:  # a baseline look only (after a restore or a capture: _auto_rebase)
                return
            frac = (walks - base[0]) / max(1, pend[1] * self.n)
            A["last_fraction"] = frac
            if frac > self.AUTO_WALK_FRACTION:
                self.cull = "cells"
                A["switched_after"] = A["steps"]
                return
        if A["pending"] is None and A["steps"] >= self.AUTO_CHECK_STEPS:
            import torch
            check(lib.cbf_lattice_window_counters(ptr(self.ws), self.ws_bytes, ptr(A["host"]), stream_handle()),
                  "cbf_lattice_window_counters")
            ev = torch.cuda.Event()
            ev.record()
            A["pending"] = (ev, A["steps"])
            A["steps"] = 0

    def _auto_rebase(self):
        """cull="auto": the workspace counters hold walks of launches _auto_check never counted (a
        restored workspace's whole history, a capture's warm-up launch), so the next look that lands
        only sets the baseline and the decision waits for the one after it."""
        if self._auto is not None:
            self._auto["base"], self._auto["pending"] = None, None

    def history(self, steps):
        """The per-timestep outputs of the last run(steps, history=True): (vel, u, status,
        nbr_count), leading dimension = timestep."""
        return self._history(steps)

    def build_phase(self):
        """nominal control + cell list only (K1-K3); window cull: nominal control + guards."""
        if self.cull == "window":
            check(lib.cbf_lattice_window_build(self.cp, _lib.C.byref(self.grid), self.W, self.H, ptr(self.pos),
                                               self.gain, ptr(self.vel), ptr(self.ws), self.ws_bytes,
                                               stream_handle()), "cbf_lattice_window_build")
            return
        check(lib.cbf_lattice_build(self.cp, _lib.C.byref(self.grid), self.W, self.H, 0, self.H, 0, self.H,
                                    ptr(self.pos), self.gain, ptr(self.vel), ptr(self.ws), self.ws_bytes,
                                    stream_handle()), "cbf_lattice_build")

    def advance_phase(self, mark=None, commit=True, timing=None):
        """filter + clip + Euler only (the dominant kernel, K4, then the queued-QP kernel K5).
        mark: a torch.cuda.Event (already recorded once) that is recorded between K4 and K5.
        timing: (start, stop) torch.cuda.Events (already recorded once) that get the filter
        kernel's own start and end times (cbf_lattice_*advance_timed, hipExtLaunchKernel).
        Window cull: the new positions go to a scratch tensor (the filter reads pos throughout) and
        are copied into pos unless commit=False (kernel timing)."""
        ev = (lambda e: _lib.C.c_void_p(e.cuda_event))
        if self.cull == "window":
            torch = _lib.require_gpu()
            if getattr(self, "_pos_next", None) is None:
                self._pos_next = torch.empty_like(self.pos)
            if timing is not None:
                check(lib.cbf_lattice_window_advance_timed(
                    self.cp, _lib.C.byref(self.grid), self.W, self.H, ptr(self.pos), self.T, ptr(self._pos_next),
                    ptr(self.u), ptr(self.status), ptr(self.nbr_count), self._st(), ptr(self.ws), self.ws_bytes,
                    ev(timing[0]), ev(timing[1]), stream_handle()), "cbf_lattice_window_advance_timed")
                if commit:
                    self.pos.copy_(self._pos_next)
                return
            check(lib.cbf_lattice_window_advance(self.cp, _lib.C.byref(self.grid), self.W, self.H, ptr(self.pos),
                                                 self.T, ptr(self._pos_next), ptr(self.u), ptr(self.status),
                                                 ptr(self.nbr_count), self._st(), ptr(self.ws), self.ws_bytes,
                                                 _lib.C.c_void_p(mark.cuda_event if mark is not None else 0),
                                                 stream_handle()), "cbf_lattice_window_advance")
            if commit:
                self.pos.copy_(self._pos_next)
            return
        if self.barrier == "euclidean_hocbf":
            check(lib.cbf_lattice_advance_hocbf(self.cp, _lib.C.byref(self.hp), _lib.C.byref(self.grid), self.W,
                                                self.H, 0, self.H, 0, self.H, ptr(self.pos), self.T, ptr(self.pos),
                                                ptr(self.u), ptr(self.status), ptr(self.nbr_count), 0, None,
                                                self._st(), ptr(self.ws), self.ws_bytes, stream_handle()),
                  "cbf_lattice_advance_hocbf")
            return
        if timing is not None:
            check(lib.cbf_lattice_advance_timed(self.cp, _lib.C.byref(self.grid), self.W, self.H, 0, self.H, 0, self.H,
                                                ptr(self.pos), self.T, ptr(self.pos), ptr(self.u), ptr(self.status),
                                                ptr(self.nbr_count), 0, None, self._st(), ptr(self.ws), self.ws_bytes,
                                                ev(timing[0]), ev(timing[1]), stream_handle()),
                  "cbf_lattice_advance_timed")
            return
        if mark is not None:
            check(lib.cbf_lattice_advance_marked(self.cp, _lib.C.byref(self.grid), self.W, self.H, 0, self.H, 0, self.H,
                                                 ptr(self.pos), self.T, ptr(self.pos), ptr(self.u), ptr(self.status),
                                                 ptr(self.nbr_count), 0, None, self._st(), ptr(self.ws), self.ws_bytes,
                                                 _lib.C.c_void_p(mark.cuda_event), stream_handle()),
                  "cbf_lattice_advance_marked")
            return
        check(lib.cbf_lattice_advance(self.cp, _lib.C.byref(self.grid), self.W, self.H, 0, self.H, 0, self.H,
                                      ptr(self.pos), self.T, ptr(self.pos), ptr(self.u), ptr(self.status),
                                      ptr(self.nbr_count), 0, None, self._st(), ptr(self.ws), self.ws_bytes,
                                      stream_handle()), "cbf_lattice_advance")

    def stats_summary(self) -> dict:
        """Rollout statistics since the last reset (host sync); raises if a step's cell list was
        unusable (CBF_STATUS_WORKSPACE_ERROR)."""
        st = _lib.decode_stats(self.stats.cpu().numpy())
        if st["errors"]:
            raise _lib.CbfError(f"{st['errors']} lattice step(s) ran on an unusable cell list (scan gave up)")
        return st

    def solves_total(self) -> int:
        return self.stats_summary()["solves"]

    def reset_solves(self):
        self.stats.zero_()

    def capture(self, steps=None, history=False):
        """Capture one step (replayed by step()) or, with `steps`, one run(steps, history) call
        (replayed by run(steps, history); one graph per step count) into a hipGraph, for the cull
        in use (cull="auto" replays it only while that cull is).  The warm-up launch outside the
        capture advances the swarm."""
        import torch
        launch = self._launch if steps is None else (lambda: self._launch_run(steps, history))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            launch()  # warm-up outside capture
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self._auto_rebase()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            launch()
        if steps is None:
            self.graphs[(self.collect_stats, self.cull)] = g
        else:
            self.run_graphs[(steps, self.collect_stats, history, self.cull)] = g
        return g

    def snapshot(self) -> list:
        """Device copies of the swarm's whole state (positions, workspace incl. the cell order and
        the nominal-control state, outputs, statistics), for restore()."""
        return [t.clone() for t in self._state()]

    def restore(self, snap: list) -> None:
        """Back to a snapshot(): the following steps repeat the snapshot's trajectory bit for bit."""
        for t, c in zip(self._state(), snap):
            t.copy_(c)

    def _state(self):
        return [self.pos, self.vel, self.u, self.status, self.nbr_count, self.ws, self.stats, self.ap_ws]

    # ---- rollout checkpoints ("save the SoA state .npz every K steps") ---------------------
    def save_checkpoint(self, path: str) -> None:
        """Write the swarm's whole device state (snapshot(): positions, nominal controls, outputs, the
        workspace with the cell order and the nominal-control spec, statistics) and what defines the
        step (shape, grid, gain, T, method, barrier, filter parameters) to an .npz.
        LatticeSwarm.from_checkpoint(path) resumes the rollout: its next steps are bit-identical to
        the ones this swarm would take.  Synchronises the device."""
        import json
        torch = _lib.require_gpu()
        torch.cuda.synchronize()
        # what the opaque workspace bytes mean: a library with another ABI, workspace layout or size
        # must not restore them (from_checkpoint refuses)
        meta = {"abi_version": int(lib.cbf_abi_version()), "workspace_layout": int(lib.cbf_workspace_layout()),
                "ws_bytes": int(self.ws_bytes),
                "W": self.W, "H": self.H, "gain": self.gain, "T": self.T, "method": self.method,
                "barrier": self.barrier, "alpha": list(self.alpha), "nominal": self.nominal, "cull": self.cull,
                "cull_mode": self.cull_mode,
                "grid": [self.grid.x0, self.grid.y0, self.grid.inv_h, self.grid.nx, self.grid.ny],
                "params": {"max_speed": self.params.max_speed, "dmin": self.params.dmin, "k": self.params.k,
                           "safety_distance": self.params.safety_distance,
                           "f": np.asarray(self.params.f, dtype=np.float64).tolist(),
                           "g": np.asarray(self.params.g, dtype=np.float64).tolist(),
                           "solve_placement": self.params.solve_placement}}
        arrays = {f"state{i}": t.cpu().numpy() for i, t in enumerate(self._state())}
        arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        with open(path, "wb") as f:
            np.savez(f, **arrays)

    @classmethod
    def from_checkpoint(cls, path: str) -> "LatticeSwarm":
        """A swarm rebuilt from save_checkpoint()'s file (no pickles: the metadata is JSON).  Steps
        and runs continue the saved rollout bit for bit; graphs are captured afresh as usual."""
        import json
        with np.load(path, allow_pickle=False) as z:
            meta = json.loads(bytes(z["meta"]).decode())
            states = [z[f"state{i}"] for i in range(8)]
        for key, have in (("abi_version", lib.cbf_abi_version()), ("workspace_layout", lib.cbf_workspace_layout())):
            if meta.get(key) != have:
                raise ValueError(f"checkpoint {path}: written with {key} {meta.get(key)}, this library has {have}: "
                                 "its workspace bytes cannot be restored")
        pr = meta["params"]
        params = FilterParams(max_speed=pr["max_speed"], dmin=pr["dmin"], k=pr["k"],
                              safety_distance=pr["safety_distance"], f=np.array(pr["f"]), g=np.array(pr["g"]),
                              solve_placement=pr.get("solve_placement", "auto"))
        g = CbfGrid()
        g.x0, g.y0, g.inv_h = (float(v) for v in meta["grid"][:3])
        g.nx, g.ny = int(meta["grid"][3]), int(meta["grid"][4])
        nominal = meta["nominal"]
        S = cls(states[0], meta["W"], meta["H"], gain=meta["gain"], params=params, T=meta["T"], grid=g,
                method=meta["method"], barrier=meta["barrier"], alpha=tuple(meta["alpha"]),
                nominal=tuple(nominal) if isinstance(nominal, list) else nominal,
                # cull="auto" resumes with the cull the saved swarm had reached
                cull="auto" if meta.get("cull_mode") == "auto" and meta.get("cull") == "window"
                else meta.get("cull", "cells"))
        if meta.get("ws_bytes") != S.ws_bytes:
            raise ValueError(f"checkpoint {path}: workspace of {meta.get('ws_bytes')} bytes, this swarm's is "
                             f"{S.ws_bytes}")
        for i, (t, a) in enumerate(zip(S._state(), states)):
            if tuple(t.shape) != a.shape or str(t.dtype).replace("torch.", "") != str(a.dtype):
                raise ValueError(f"checkpoint {path}: state{i} does not fit this swarm ({a.shape}, {a.dtype} vs "
                                 f"{tuple(t.shape)}, {t.dtype})")
            t.copy_(_lib.require_gpu().from_numpy(a))
        S._auto_rebase()  # the restored workspace carries the saved rollout's walk counts
        return S

    def step(self):
        g = self.graphs.get((self.collect_stats, self.cull))
        if g is not None:
            g.replay()
        else:
            self._launch()
        self._auto_check(1)


def mc_rollout(params, pos, n_o, n_a, steps, T=1 / 30, theta=None, so=1.0, ga=1.0, safety=False, stats=True):
    """SURVEY cfg5: pos (n_scen, n_o+n_a, 2) CUDA float64, advanced in place by `steps` steps.
    Returns (counters int64 (n_scen,4) = {filter calls, relaxed, box-infeasible, relax-cap},
    maxviol (n_scen,) = max row violation over OPTIMAL solves[, safety (n_scen, 2) = {max violation
    of the original barrier rows over RELAXED solves, min neighbour distance^2}]).  stats=False:
    the kernel instantiation without statistics (maxviol / safety are None; same positions and
    counters)."""
    torch = _lib.require_gpu()
    theta = -math.pi / n_o if theta is None else theta
    rc, rs = float(np.cos(theta)), float(np.sin(theta))
    n_scen = pos.shape[0]
    assert pos.is_contiguous() and pos.dtype == torch.float64 and pos.shape[1] == n_o + n_a
    cnt = torch.empty((n_scen, 4), dtype=torch.int64, device=pos.device)
    mv = torch.empty((n_scen,), dtype=torch.float64, device=pos.device) if stats else None
    sf = torch.empty((n_scen, 2), dtype=torch.float64, device=pos.device) if safety and stats else None
    cp = params.c() if isinstance(params, FilterParams) else params
    check(lib.cbf_mc_rollout(cp, n_scen, n_o, n_a, steps, float(T), rc, rs, float(so), float(ga), ptr(pos), ptr(cnt),
                             ptr(mv), ptr(sf), stream_handle()), "cbf_mc_rollout")
    return (cnt, mv, sf) if safety else (cnt, mv)
