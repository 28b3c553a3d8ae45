# Round-4 final pass, part 2: the headline's kernel trace + stats, a 3-step timeline and the
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${FINAL_TAG:-r04f}
PROF_TAG=$T bash scripts/gpu_profile.sh || exit $?
TL_TAG=$T bash scripts/gpu_timeline.sh > gpurun_out/timeline_$T.txt || exit $?
PROF_TAG=$T PMC_MORE=0 bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_$T > gpurun_out/pmc_${T}_summary.json 2> gpurun_out/pmc_${T}_summary.err || true
