# Build an A/B tree tools/_abt/<name> from a git revision's cbf_amd/ and include/ (default HEAD),
# with optional extra -D switches.   Usage: bash tools/mk_ab_head.sh <name> [rev] ["DEF1=1 ..."]
set -e
cd "$(dirname "$0")/.."
T=tools/_abt/$1; REV=${2:-HEAD}
rm -rf $T && mkdir -p $T
git archive $REV cbf_amd include | tar -x -C $T
CBF_EXTRA_DEFS="${3:-}" python -c "import sys; sys.path.insert(0, '$T'); import importlib.util as u; s = u.spec_from_file_location('b', '$T/cbf_amd/build.py'); m = u.module_from_spec(s); s.loader.exec_module(m); m.build()"
echo "built $T ($REV ${3:-})"
