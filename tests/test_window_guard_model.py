"""The lattice-window cull's completeness argument (cbf_amd/csrc/window.hip), checked on the CPU
with a numpy model of its guards: for every ego, the candidates the window cull tests -- the rows
of its row guard, columns c-1..c+1 (c-+2 where a sentinel fails), or the unbounded walk -- contain
every agent that passes the reference's cull test s < 0.04, s > 0 (cross_and_rescue.py:141-150).
The GPU tests compare the kernel with the oracle; this one exercises the argument itself on swarms
far less lattice-like than any rollout (random shuffles, folded rows, clumps, non-finite values)."""
import numpy as np
import pytest

CULL_T = 0.2 * 0.2


def _win_d(cull_t):
    d = np.sqrt(cull_t)
    while d * d < cull_t:
        d = np.nextafter(d, np.inf)
    return d


def _f32_down(v):
    f = v.astype(np.float32)
    bad = f.astype(np.float64) > v
    f[bad] = np.nextafter(f[bad], np.float32(-np.inf))
    return f


def _f32_up(v):
    f = v.astype(np.float32)
    bad = f.astype(np.float64) < v
    f[bad] = np.nextafter(f[bad], np.float32(np.inf))
    return f


def _guards(pos, W, H):
    """k_window_prep's outputs: sylo, pyhi per row, (rs, rp) per agent, over finite agents."""
    x = pos[:, 0].reshape(H, W)
    y = pos[:, 1].reshape(H, W)
    fin = np.isfinite(x) & np.isfinite(y)
    ylo = np.where(fin, y, np.inf).min(axis=1)
    yhi = np.where(fin, y, -np.inf).max(axis=1)
    sylo = np.append(np.minimum.accumulate(ylo[::-1])[::-1], np.inf)
    pyhi = np.maximum.accumulate(yhi)
    xs = np.where(fin, x, np.inf)
    rs = np.minimum.accumulate(xs[:, ::-1], axis=1)[:, ::-1]
    xp = np.where(fin, x, -np.inf)
    rp = np.maximum.accumulate(xp, axis=1)
    return sylo, pyhi, _f32_down(rs).astype(np.float64), _f32_up(rp).astype(np.float64)


def _tested(pos, W, H, e, G, d):
    """The window indices the window cull tests for ego e: k_window_tile's candidates (rows of the
    row guard, columns c-1..c+1, c-+2 where a sentinel fails) or, where that is not enough, the
    unbounded walk of win_direct."""
    sylo, pyhi, rs, rp = G
    r, c = divmod(e, W)
    xe, ye = pos[e]
    if not (np.isfinite(xe) and np.isfinite(ye)):
        return set()   # no candidate can pass
    ku = 0
    while r + ku + 1 < H and not (sylo[r + ku + 1] - ye > d):
        ku += 1
    kd = 0
    while r - kd - 1 >= 0 and not (ye - pyhi[r - kd - 1] > d):
        kd += 1
    out = set()
    slow = False
    for dr in range(-kd, ku + 1):
        rr = r + dr
        cols = [cc for cc in (c - 1, c, c + 1) if 0 <= cc < W]
        right = c + 2 >= W or rs[rr, c + 2] - xe > d
        left = c - 2 < 0 or xe - rp[rr, c - 2] > d
        if not right:
            cols.append(c + 2)
            if not (c + 3 >= W or rs[rr, c + 3] - xe > d):
                slow = True
        if not left:
            cols.append(c - 2)
            if not (c - 3 < 0 or xe - rp[rr, c - 3] > d):
                slow = True
        out.update(rr * W + cc for cc in cols)
    if slow:   # win_direct: every row walked outward until its sentinels hold
        out = set()
        for dr in range(-kd, ku + 1):
            rr = r + dr
            cc = c
            while cc < W:
                out.add(rr * W + cc)
                if cc + 1 >= W or rs[rr, cc + 1] - xe > d:
                    break
                cc += 1
            cc = c - 1
            while cc >= 0:
                out.add(rr * W + cc)
                if cc - 1 < 0 or xe - rp[rr, cc - 1] > d:
                    break
                cc -= 1
    return out


def _check(pos, W, H):
    d = _win_d(CULL_T)
    G = _guards(pos, W, H)
    n = W * H
    with np.errstate(invalid="ignore", over="ignore"):
        for e in range(n):
            e0 = pos[:, 0] - pos[e, 0]
            e1 = pos[:, 1] - pos[e, 1]
            s = (0.0 + e0 * e0) + e1 * e1
            nbrs = set(np.nonzero((s < CULL_T) & (s > 0))[0].tolist())
            miss = nbrs - _tested(pos, W, H, e, G, d)
            assert not miss, (e, sorted(miss))


def _lattice(W, H, rng, a=0.145):
    r, c = np.divmod(np.arange(W * H), W)
    p = np.stack([c * a, r * a], axis=1).astype(np.float64)
    return p + rng.uniform(-a / 2, a / 2, size=p.shape)


@pytest.mark.parametrize("seed", range(4))
def test_window_guards_complete_on_jittered_lattices(seed):
    rng = np.random.default_rng(seed)
    W, H = 24, 18
    _check(_lattice(W, H, rng, a=rng.uniform(0.1, 0.25)), W, H)


@pytest.mark.parametrize("seed", range(4))
def test_window_guards_complete_on_scrambled_swarms(seed):
    rng = np.random.default_rng(100 + seed)
    W, H = 20, 16
    pos = _lattice(W, H, rng)
    k = rng.integers(5, 60)
    a, b = rng.choice(W * H, k, replace=False), rng.choice(W * H, k, replace=False)
    pos[a], pos[b] = pos[b].copy(), pos[a].copy()
    clump = rng.choice(W * H, 12, replace=False)
    pos[clump] = rng.uniform(0.5, 0.7, size=(12, 2))
    pos[rng.integers(W * H)] = pos[rng.integers(W * H)]
    _check(pos, W, H)


def test_window_guards_complete_on_folded_and_random_swarms():
    rng = np.random.default_rng(7)
    W, H = 16, 12
    pos = _lattice(W, H, rng).reshape(H, W, 2)
    pos[1::2] = pos[1::2, ::-1]              # rows out of x order
    pos[3], pos[9] = pos[9].copy(), pos[3].copy()   # rows out of y order
    _check(pos.reshape(-1, 2).copy(), W, H)
    _check(rng.uniform(0, 1.0, size=(W * H, 2)), W, H)   # no lattice structure at all


def test_window_guards_complete_with_nonfinite_positions():
    rng = np.random.default_rng(8)
    W, H = 16, 10
    pos = _lattice(W, H, rng)
    pos[5] = [np.nan, 0.3]
    pos[40] = [np.inf, pos[40, 1]]
    pos[77] = [pos[77, 0], -np.inf]
    _check(pos, W, H)


def test_window_margin_is_exact():
    """win_d: the smallest double whose square is >= cull_t, so a coordinate difference beyond it
    cannot pass s < cull_t (rounding is monotone)."""
    d = _win_d(CULL_T)
    assert d * d >= CULL_T and np.nextafter(d, 0) ** 2 < CULL_T
