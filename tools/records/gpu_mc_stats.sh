# GPU box: the statistics-free Monte-Carlo kernel: MC GPU tests, cfg5 profile and bench line
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/mcst; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "mc_rollout" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PROF_OUT=$O/prof CONFIGS=cfg5 bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 2; }
timeout -k 10 400 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 3; }
python -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'], d['ms_per_step_with_stats'], d['safety'])"
