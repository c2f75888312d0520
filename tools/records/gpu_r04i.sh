# GPU box, round 4: kernel traces and PMC passes of cfg4 / cfg4f (window cull) and cfg4r (cell
# list) with the current kernel names (tools/profile.sh), for profiles/pmc_summary.json.
set -u
cd "$GRAFT_REPO_ROOT"
PROF_OUT=gpurun_out/prof_r04 CONFIGS="cfg4 cfg4f cfg4r" bash tools/profile.sh || exit 1
echo R04I_OK
