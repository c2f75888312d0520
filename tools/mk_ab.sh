# Build an A/B variant tree tools/_abt/<name> (git-ignored; sent to the GPU box, unlike tools/_ab) (a copy of cbf_amd/ and include/) with extra -D switches.
# Usage: bash tools/mk_ab.sh <name> "DEF1=1 DEF2=3"
set -e
cd "$(dirname "$0")/.."
T=tools/_abt/$1
rm -rf $T && mkdir -p $T
cp -r cbf_amd include $T/
rm -rf $T/cbf_amd/_build $T/cbf_amd/*.so
CBF_EXTRA_DEFS="$2" python -c "import sys; sys.path.insert(0, '$T'); import importlib.util as u; s = u.spec_from_file_location('b', '$T/cbf_amd/build.py'); m = u.module_from_spec(s); s.loader.exec_module(m); m.build()"
echo "built $T ($2)"
