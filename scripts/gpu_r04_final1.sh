# Round-4 final pass, part 1: GPU suite, smoke, the default bench line (every leg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${FINAL_TAG:-r04_final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/${T}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 bench.py > gpurun_out/${T}_bench.json.log 2>&1
rc=$?; echo bench_rc=$rc
tail -c 400 gpurun_out/${T}_bench.json.log
exit $rc
