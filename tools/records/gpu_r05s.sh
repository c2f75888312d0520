# GPU box: the tile's staged column halo (kTileKC 3 / 5 / 8: the window walk's LDS reach): the
# driver's bench line and run(10), interleaved.
set -u
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu/gpu_r05k.sh tools/_abt/base tools/_abt/kc5 tools/_abt/kc8 || exit 2
for rep in 1 2; do
  for t in tools/_abt/base tools/_abt/kc5 tools/_abt/kc8; do
    timeout -k 10 120 python3 tools/ab_window.py $t window 0.145 || exit 3
  done
done
