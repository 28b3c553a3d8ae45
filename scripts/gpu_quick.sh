#!/bin/bash
# Quick GPU iteration: the GPU tests (stop at the first failure), then the headline bench
# with its full-size check but no legs. Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --legs "${LEGS:-}" ${BENCH_ARGS:-} \
    > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
exit $rc
