"""Filter parameter sets for the fused-path oracle tests.

The reference's filter takes max_speed / dmin / k in its constructor (cbf.py:6) and the dynamics
f, g in every call (cbf.py:55-59); its callers pass max_speed 15, dmin 0.2, k 1, f = 0 and
g = 0.1 [I2; 0] (cross_and_rescue.py:30-32) and cull at 0.2 (:134).  The golden fixtures pin the
row arithmetic at other values (tests/golden/make_golden.py tags 6-8); these sets run the fused
kernels (lattice, window, Monte-Carlo, swarm filters) at such values against the oracle, which
executes their f != 0 instantiations and, with the wider cull radius, the window cull's
beyond-the-tile walk.
"""
import numpy as np

_rng = np.random.default_rng(20261018)
F_RAND = np.round(_rng.normal(0, 0.5, (4, 4)), 6)
G_RAND = np.round(_rng.normal(0, 0.3, (4, 2)), 6)
F_RAND2 = np.round(_rng.normal(0, 0.2, (4, 4)), 6)

CALLERS_G = 0.1 * np.array([[1, 0], [0, 1], [0, 0], [0, 0]])

SETS = {
    # the callers' constants (cross_and_rescue.py:30-32,134)
    "callers": dict(max_speed=15.0, dmin=0.2, k=1.0, safety_distance=0.2, f=np.zeros((4, 4)), g=CALLERS_G),
    # every parameter away from its default at once
    "nondefault": dict(max_speed=2.0, dmin=0.35, k=2.0, safety_distance=0.3, f=F_RAND, g=G_RAND),
    # non-integer k (hs_p a float array), f != 0, the callers' g and radius
    "kfrac": dict(max_speed=15.0, dmin=0.2, k=1.5, safety_distance=0.2, f=F_RAND2, g=CALLERS_G),
}
NAMES = list(SETS)


def filter_params(name, **kw):
    from cbf_amd import swarm
    return swarm.FilterParams(**SETS[name], **kw)


def oracle_params(name):
    from oracle import pyoracle as po
    s = SETS[name]
    return po.Params(s["max_speed"], s["dmin"], s["k"], f=s["f"], g=s["g"], safety_distance=s["safety_distance"])
