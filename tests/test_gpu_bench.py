"""bench.py's output contract on the GPU: stdout is exactly one JSON line with the fields the
driver reads, also when RCCL is initialised (its version banner must not reach stdout)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _bench(*args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--width", "256", "--rows", "256",
                        "--steps", "3", "--warmup", "1", "--kernel-iters", "2", "--no-cpu-baseline", *args],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert KEYS <= set(res)
    assert res["value"] > 0 and res["n_gpus"] == 1 and res["steps"] == 3
    return res


@pytest.mark.gpu
def test_bench_single_gpu_one_json_line():
    res = _bench()
    assert res["config"]["graph"] is True
    assert res["roofline"]["bound"] == "hbm" and res["roofline"]["achieved"] > 0


@pytest.mark.gpu
def test_bench_sharded_rccl_one_json_line():
    res = _bench("--shard")  # RCCL communicator of one rank: the sharded step with its collective
    assert "RCCL" in res["config"]["parallelism"]
