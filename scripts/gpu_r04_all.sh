# Suite (stops at the first failure), then the round-4 evidence pass (kernel trace, timeline,
# PMC) of the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${SUITE_TAG:-x}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
PROF_TAG=${PROF_TAG:-r04j} bash scripts/gpu_r04_prof.sh
