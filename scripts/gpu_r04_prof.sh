# Round-4 evidence pass: kernel trace + stats of the headline, a 3-step timeline, and the
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, TCC) of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF_TAG=${PROF_TAG:-r04a} bash scripts/gpu_profile.sh || exit $?
TL_TAG=${PROF_TAG:-r04a} TL_STEPS=3 bash scripts/gpu_timeline.sh > gpurun_out/timeline_${PROF_TAG:-r04a}.txt || exit $?
PROF_TAG=${PROF_TAG:-r04a} bash scripts/gpu_pmc.sh || exit $?
