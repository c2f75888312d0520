# GPU box, round 3: block-staged candidate rows in the lattice filter (tools/_ab/st256, st384:
# CBF_STAGE=1 with 256 / 384 slots per row segment) and the restructured unstaged filter (this
# tree, CBF_STAGE=0) against the committed tree (tools/_ab/base): lattice parity tests of each
# staged build (through CBF_LIB), A/B, kernel traces at cfg4.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03st; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k lattice > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
(cd tools/_ab/st256 && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k lattice) > $O/pytest_st256.log 2>&1 || { tail -40 $O/pytest_st256.log; exit 1; }
tail -1 $O/pytest_st256.log
for t in tools/_ab/st256 tools/_ab/st384; do
  n=$(basename $t)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 3
done
for rep in 1 2; do
  for t in . tools/_ab/st256 tools/_ab/st384 tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
echo R03ST_OK
