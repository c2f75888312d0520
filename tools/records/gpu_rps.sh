# GPU box: rps-lite parity tests, then the certificate bench at N = 16, 4, 32
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rps_tests.log 2>&1 || { tail -30 gpurun_out/rps_tests.log; exit 1; }
tail -2 gpurun_out/rps_tests.log
bash tools/gpu_cert.sh
