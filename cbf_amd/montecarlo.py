"""Batched Monte-Carlo rendezvous (SURVEY cfg5, meet_at_center.py:76-153 per scenario), scenarios
sharded across ranks: rank r of W owns the contiguous scenario range
[r * ceil(S / W), ...) and rolls it out with no per-step communication; the totals are combined
by one all-reduce per quantity at the end (counts summed, violations maxed, distances minned).

The backend does the device work: HipBackend (cbf_mc_rollout on the rank's GPU) in production;
the CPU gloo tests plug in the oracle as a backend to check the sharding and reduction logic.
"""
from __future__ import annotations

import math

import numpy as np

from . import scenarios


def shard_bounds(n_scen: int, world: int, rank: int):
    """Contiguous scenario range [lo, hi) of `rank` out of `world` (the last ranks may be short)."""
    per = (n_scen + world - 1) // world
    lo = min(n_scen, rank * per)
    return lo, min(n_scen, lo + per)


class HipBackend:
    """cbf_mc_rollout on the current GPU (swarm.mc_rollout)."""

    def __init__(self, params=None):
        import torch
        from . import swarm
        self.torch, self.swarm = torch, swarm
        self.params = params or swarm.FilterParams()

    def tensor(self, a):
        return self.torch.as_tensor(np.ascontiguousarray(a), device="cuda")

    def rollout(self, pos, n_o, n_a, steps, ga, stats=True):
        """Advances pos in place; returns (counters (B,4) int64, maxviol (B,), safety (B,2)); with
        stats=False the last two are None (the kernel without statistics)."""
        return self.swarm.mc_rollout(self.params, pos, n_o, n_a, steps, ga=ga, safety=True, stats=stats)


class MonteCarlo:
    """This rank's shard of an n_scen-scenario batch of n_o + n_a rendezvous scenarios."""

    def __init__(self, n_scen, n_o=16, n_a=16, seed=0, ga=scenarios.MC_GAIN, backend=None, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        self.n_scen, self.n_o, self.n_a, self.ga = n_scen, n_o, n_a, ga
        self.lo, self.hi = shard_bounds(n_scen, self.world, self.rank)
        self.be = backend or HipBackend()
        # scenario s's initial condition depends only on (seed, s), whatever the sharding
        self.pos = self.be.tensor(scenarios.mc_scenarios(n_scen, n_o, n_a, seed=seed)[self.lo:self.hi])
        # False: the rollouts compute no violations or distances (counters only), bit-identical
        self.collect_stats = True
        self.reset_totals()

    def reset_totals(self):
        self.counts = np.zeros(4, np.int64)          # filter calls, relaxed, box-infeasible, relax-cap
        self.viol_opt = 0.0                          # max row violation over OPTIMAL solves
        self.viol_orig = 0.0                         # max original-row violation over RELAXED solves
        self.min_d2 = math.inf                       # min neighbour distance^2
        # running accumulators of the rollouts since the last fold, in the backend's array type
        # (device tensors for the HIP backend): each rollout's per-scenario results are reduced
        # into them right away (no host sync), so a long run holds O(1) result memory
        self._acc = None

    def _fold(self, cnt, mv, sf):
        """Reduce one rollout's per-scenario results into the running accumulators: counts summed,
        {max violation (OPTIMAL), max original-row violation (RELAXED), -min distance^2} maxed."""
        xp = np
        if hasattr(cnt, "is_cuda"):
            import torch as xp
        c = cnt.sum(0)
        # (the backends return both statistics arrays or neither)
        m = None if mv is None or sf is None else xp.stack([mv.max(), sf[:, 0].max(), -sf[:, 1].min()])
        if self._acc is None:
            self._acc = [c, m]
            return
        self._acc[0] = self._acc[0] + c
        if m is not None:
            self._acc[1] = m if self._acc[1] is None else xp.maximum(self._acc[1], m)

    def run(self, steps):
        """Advance this rank's scenarios by `steps` timesteps (device work only; no host sync)."""
        if self.hi > self.lo:
            self._fold(*(self.be.rollout(self.pos, self.n_o, self.n_a, steps, self.ga) if self.collect_stats
                         else self.be.rollout(self.pos, self.n_o, self.n_a, steps, self.ga, stats=False)))

    def snapshot(self):
        """A copy of this rank's scenario states, for restore()."""
        return self.pos.clone()

    def restore(self, snap):
        """Back to a snapshot(): the following runs repeat its rollouts bit for bit."""
        self.pos.copy_(snap)

    def _local(self):
        if self._acc is not None:
            c, m = self._acc
            self.counts += np.asarray(c.tolist(), dtype=np.int64)
            if m is not None:
                m = [float(v) for v in m.tolist()]
                self.viol_opt = max(self.viol_opt, m[0])
                self.viol_orig = max(self.viol_orig, m[1])
                self.min_d2 = min(self.min_d2, -m[2])
        self._acc = None

    def totals(self) -> dict:
        """The whole batch's counters and safety record (one all-reduce per kind across ranks)."""
        import torch
        self._local()
        c = torch.tensor(self.counts, dtype=torch.int64)
        m = torch.tensor([self.viol_opt, self.viol_orig], dtype=torch.float64)
        d = torch.tensor([self.min_d2], dtype=torch.float64)
        if self.world > 1:
            if self.dist.get_backend(self.group) == "nccl":
                c, m, d = c.cuda(), m.cuda(), d.cuda()
            self.dist.all_reduce(c, group=self.group)
            self.dist.all_reduce(m, op=self.dist.ReduceOp.MAX, group=self.group)
            self.dist.all_reduce(d, op=self.dist.ReduceOp.MIN, group=self.group)
        c, m, d = c.cpu().numpy(), m.cpu().numpy(), float(d.cpu()[0])
        calls = int(c[0])
        return {"calls": calls, "relaxed": int(c[1]), "box_infeasible": int(c[2]), "relax_cap": int(c[3]),
                "feasible_fraction": (calls - int(c[1:].sum())) / max(calls, 1),
                "max_violation_optimal": float(m[0]), "max_violation_original_rows_relaxed": float(m[1]),
                "min_pairwise_distance": math.sqrt(d) if math.isfinite(d) else None}
