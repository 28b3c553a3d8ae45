# Full GPU test suite (one process, stops at the first failure), then the default bench.
mkdir -p gpurun_out
T=${SUITE_TAG:-x}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -c 600 gpurun_out/${T}_bench.log
exit $rc
