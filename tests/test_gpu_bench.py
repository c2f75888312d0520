"""bench.py's output contract on the GPU: stdout is exactly one JSON line with the fields the
driver reads, also when RCCL is initialised (its version banner must not reach stdout), and
`--gpus N` without a launcher starts N ranks itself (strong scaling by default: the same lattice
split N ways, ending in the same state as the 1-rank run)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _bench(*args, n=1, steps=3):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--width", "256", "--rows", "256",
                        "--steps", str(steps), "--warmup", "1", "--kernel-iters", "2", "--no-cpu-baseline", *args],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert KEYS <= set(res)
    assert res["value"] > 0 and res["n_gpus"] == n and res["steps"] == steps
    return res


@pytest.mark.gpu
def test_bench_single_gpu_one_json_line():
    res = _bench()
    assert res["config"]["graph"] is True
    assert res["roofline"]["bound"] == "hbm" and res["roofline"]["achieved"] > 0
    assert res["ms_per_step_outputs_every_step"] > 0   # the per-step-outputs replay ran and matched


@pytest.mark.gpu
def test_bench_sharded_rccl_one_json_line():
    res = _bench("--shard")  # RCCL communicator of one rank: the sharded step with its collective
    assert "single-rank" in res["config"]["parallelism"] and "all-to-all" in res["config"]["parallelism"]


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks_strong_scaling():
    """`bench.py --gpus 2` (no torchrun) runs two ranks (gloo here: one GPU on this box), reports
    n_gpus 2 over the SAME 256 x 256 lattice (strong scaling), and ends in the state of the 1-rank
    run of the same timesteps, bit for bit (sha256 of all positions)."""
    one = _bench(steps=10)
    two = _bench("--gpus", "2", "--backend", "gloo", n=2, steps=10)
    assert two["config"]["agents_total"] == one["config"]["agents_total"] == 256 * 256
    assert two["config"]["agents_per_gpu"] == 256 * 128
    assert two["scaling"] == "strong" and "x2" in two["config"]["parallelism"]
    assert two["end_state_sha256"] == one["end_state_sha256"]
    assert two["solves_per_step"] == one["solves_per_step"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 8])
def test_bench_gpus_n_rehearsal_matches_one_rank(n):
    """The 4- and 8-rank row splits of the strong-scaling bench (64 and 32 rows per rank of a
    256 x 256 lattice: interior ranks with two neighbours, fewer sub-steps per exchange), rehearsed
    with gloo on this one-GPU box (8 processes on the card), end in the 1-rank state bit for bit."""
    one = _bench(steps=8)
    many = _bench("--gpus", str(n), "--backend", "gloo", n=n, steps=8)
    assert many["config"]["agents_total"] == 256 * 256
    assert many["config"]["agents_per_gpu"] == 256 * 256 // n
    assert many["end_state_sha256"] == one["end_state_sha256"]
    assert many["solves_per_step"] == one["solves_per_step"]
