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
def test_bench_gpus2_window_cull_matches_one_rank():
    """Stripes of 256 rows per rank take the window cull by default (bench.lattice_cull): the
    2-rank split of a 256 x 512 lattice (gloo, this one GPU) ends in the 1-rank state bit for
    bit."""
    one = _bench("--rows", "512", steps=6)
    two = _bench("--gpus", "2", "--backend", "gloo", "--rows", "512", n=2, steps=6)
    assert one["config"]["cull"] == "window" and two["config"]["cull"] == "window"
    assert two["config"]["agents_per_gpu"] == 256 * 256
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


@pytest.mark.gpu
def test_bench_rank_failure_is_named_and_fails_fast():
    """`bench.py --gpus 2` (gloo, one GPU) with rank 1 killed (SIGKILL) in its timed region: the
    launcher names rank 1 as the first failure at once, relays every rank's stderr with a rank
    prefix, and exits non-zero within the grace period instead of waiting on rank 0, which is left
    blocked in (or failing out of) the next collective."""
    import re
    import signal
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    grace = 20
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--width", "256", "--rows", "256",
                          "--steps", "20000", "--warmup", "1", "--kernel-iters", "2", "--no-cpu-baseline",
                          "--gpus", "2", "--backend", "gloo", "--rank-grace", str(grace),
                          "--collective-timeout", "60"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    seen, victim, t_kill = [], None, None
    t0 = time.time()
    try:
        for line in p.stderr:
            seen.append(line)
            m = re.search(r"^\[rank 1\] bench\.py rank 1/2 \(pid (\d+)\): cfg4: timed region \(", line)
            if m:
                victim = int(m.group(1))
                os.kill(victim, signal.SIGKILL)
                t_kill = time.time()
                break
            if time.time() - t0 > 150:
                break
        assert victim is not None, "".join(seen)[-3000:]
        out, err = p.communicate(timeout=grace + 90)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    err = "".join(seen) + err
    assert p.returncode != 0 and out.strip() == "", (p.returncode, out[-500:])
    assert time.time() - t_kill < grace + 60
    assert "rank 1 failed first (signal 9)" in err, err[-3000:]
    assert "FAILED: rank exit codes" in err and "first failure: rank 1" in err, err[-3000:]
    assert "[rank 0] bench.py rank 0/2" in err        # rank 0's stderr is relayed with its prefix
