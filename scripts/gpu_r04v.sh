# Current-build evidence: a 3-step kernel timeline of the headline and its HBM counter
# passes (FETCH_SIZE, WRITE_SIZE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TL_TAG=r04v bash scripts/gpu_timeline.sh > gpurun_out/timeline_r04v.txt || exit $?
PROF_TAG=r04v PMC_MORE=0 bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_r04v > gpurun_out/pmc_r04v_summary.log 2>&1 || true
