"""Synthetic workloads of BASELINE.json / SURVEY.md 8(d), as plain numpy initial conditions.

cfg1  cross_and_rescue.py as shipped (geometry :36-57, Laplacians :79-95), single-integrator
      robots (rps unavailable: documented deviation)
cfg2  meet_at_center.py (geometry :37-48, Laplacians :65-74) at N=10 (shipped) and N=100
      (complete-graph gain 4/49)
cfg3  N=65,536 jittered lattice (256 x 256, spacing 0.145), all-pairs cull
cfg4  N=1,048,576 jittered lattice (1024 x 1024), cell-list cull; sharded in row stripes
cfg5  100k independent 16+16 rendezvous scenarios (radius 0.7 / 1.05, random rotation + jitter)
"""
from __future__ import annotations

import numpy as np

T = 1 / 30                      # cross_and_rescue.py:68
LATTICE_SPACING = 0.145
LATTICE_GAIN = 0.25


def cross_and_rescue():
    """Entities: 6 pursuit obstacles, the static origin obstacle, 4 robots (cross_and_rescue.py:36-57,
    :130-133).  Returns (pos (11,2), n_obs, groups) for swarm.GroupSwarm."""
    N_robots, N_obs, diameter = 4, 6, 0.6
    ic_r = np.zeros((N_robots, 3)); ic_o = np.zeros((N_obs, 2))
    center_obs = np.array([0, 0]); center_robots = np.array([0, 0, 0])
    for i in range(N_obs):
        theta = i * (2 * np.pi / N_obs)
        ic_o[i] = center_obs + [diameter * np.cos(theta), diameter * np.sin(theta)]
    for i in range(N_robots):
        theta = i * (2 * np.pi / N_robots)
        ic_r[i] = center_robots + [0.6 * diameter * np.cos(theta) - 1.15, 0.6 * diameter * np.sin(theta),
                                   theta + (2 / 3 * np.pi)]
    pos = np.concatenate([ic_o, np.zeros((1, 2)), ic_r[:, :2]])
    ring = [[(i + 1) % N_obs] for i in range(N_obs)]                       # L1, :79-86
    l2 = [[4], [0, 3], [0, 1], [0, 2]]                                      # L2 rows 0..3, :89-95 (col 4 = goal)
    th = -np.pi / N_obs
    groups = [(0, 6, ring, None, (np.cos(th), np.sin(th)), 0.05),
              (7, 11, l2, np.array([[1.5, 0.0]]), None, 1.0)]
    return pos, 7, groups


def meet_at_center(N=10, gain=None):
    """meet_at_center.py:31-74 generalised to N (N/2 pursuit obstacles, N/2 free agents)."""
    half = N // 2
    diameter = 0.7
    ic = np.zeros((N, 3)); center = np.array([0, 0, 0])
    for i in range(half):
        theta = i * (2 * np.pi / half)
        ic[i] = center + [diameter * np.cos(theta), diameter * np.sin(theta), theta + (2 / 3 * np.pi)]
    for i in range(half, N):
        theta = i * (2 * np.pi / half) + np.pi / 5
        ic[i] = center + [1.5 * diameter * np.cos(theta), 1.5 * diameter * np.sin(theta), theta + (2 / 3 * np.pi)]
    if gain is None:
        gain = 1.0 if N == 10 else 4 / (half - 1)
    ring = [[(i + 1) % half] for i in range(half)]
    full = [[j for j in range(half) if j != i] for i in range(half)]
    th = -np.pi / half
    groups = [(0, half, ring, None, (np.cos(th), np.sin(th)), 1.0),
              (half, N, full, None, None, gain)]
    return ic[:, :2].copy(), half, groups


def lattice(W, H, seed=0, spacing=LATTICE_SPACING):
    """Jittered W x H lattice (row-major, row r at y = r*spacing), jitter U(-a/2, a/2)."""
    rng = np.random.default_rng(seed)
    r, c = np.divmod(np.arange(W * H), W)
    pos = np.stack([c * spacing, r * spacing], axis=1).astype(np.float64)
    pos += rng.uniform(-spacing / 2, spacing / 2, size=pos.shape)
    return pos


def mc_scenarios(n_scen, n_o=16, n_a=16, seed=0, r_o=0.7, r_a=1.05, jitter=0.02):
    """cfg5 initial conditions: (n_scen, n_o+n_a, 2).  Scenario s is rotated by U[0, 2pi) and
    jittered by N(0, jitter^2) per coordinate."""
    rng = np.random.default_rng(seed)
    phi = rng.uniform(0, 2 * np.pi, size=(n_scen, 1))
    th_o = np.arange(n_o) * (2 * np.pi / n_o)
    th_a = np.arange(n_a) * (2 * np.pi / n_a) + np.pi / n_a
    ang = np.concatenate([th_o[None, :] + phi, th_a[None, :] + phi], axis=1)
    rad = np.concatenate([np.full(n_o, r_o), np.full(n_a, r_a)])[None, :]
    pos = np.stack([rad * np.cos(ang), rad * np.sin(ang)], axis=2)
    pos += rng.normal(0.0, jitter, size=pos.shape)
    return np.ascontiguousarray(pos)


MC_GAIN = 4 / 15  # complete-graph gain for 16 free agents
