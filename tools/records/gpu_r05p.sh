# GPU box (diagnostic): the window tile with and without its (rare) walk code in the timed
# instantiation -- run(10) timings by tools/ab_window.py (the walk-free tree's results are wrong).
set -u
cd /root/repo
export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in tools/_abt/base tools/_abt/diagskip tools/_abt/diagcode; do
    timeout -k 10 120 python3 tools/ab_window.py $t window 0.145 || exit 1
  done
done
