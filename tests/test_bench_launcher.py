"""bench.py's rank launcher (--gpus N without torchrun) on the CPU: ranks that cannot run (no GPU in
this container) are reported by rank, with their stderr relayed under a rank prefix, and the
launcher exits non-zero -- it never waits on them forever."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_names_failed_ranks_and_exits_nonzero():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""     # no device even on a GPU box: every rank fails at set-up
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--width", "64", "--rows", "64", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--rank-grace", "10", "--rank-timeout", "240"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert time.time() - t0 < 240
    assert "failed first" in r.stderr and "FAILED: rank exit codes" in r.stderr, r.stderr[-3000:]
    assert "[rank 0] " in r.stderr and "[rank 1] " in r.stderr, r.stderr[-3000:]


def test_default_rank_timeout_is_bounded():
    sys.path.insert(0, ROOT)
    import argparse
    import bench
    a = argparse.Namespace(steps=200, warmup=20, collective_timeout=300.0)
    t = bench.default_rank_timeout(a)
    assert 300 < t < 1800


def test_lattice_cull_policy():
    """bench.py --cull auto: the window cull for the consensus lattice on one GPU and for sharded
    stripes of >= 256 rows per rank; the cell list otherwise."""
    sys.path.insert(0, ROOT)
    import argparse
    import pytest
    import bench

    def a(**kw):
        d = dict(barrier="reference", width=1024, cull="auto", nominal=None)
        d.update(kw)
        return argparse.Namespace(**d)
    assert bench.lattice_cull(a(), sharded=False) == "window"
    assert bench.lattice_cull(a(), sharded=True, rows=128) == "cells"    # N = 8 share of 1024 rows
    assert bench.lattice_cull(a(), sharded=True, rows=256) == "window"   # N = 4
    assert bench.lattice_cull(a(), sharded=True, rows=1024) == "window"  # weak scaling
    assert bench.lattice_cull(a(nominal=("random", 1.0, 5)), sharded=False) == "cells"
    assert bench.lattice_cull(a(barrier="euclidean_hocbf"), sharded=False) == "cells"
    assert bench.lattice_cull(a(width=4096), sharded=False) == "cells"
    assert bench.lattice_cull(a(cull="window"), sharded=True) == "window"
    assert bench.lattice_cull(a(cull="cells"), sharded=False) == "cells"
    with pytest.raises(SystemExit):
        bench.lattice_cull(a(cull="window", barrier="euclidean_hocbf"), sharded=False)
