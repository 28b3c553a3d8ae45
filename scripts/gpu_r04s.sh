# Limiter tests, sharded kernels, the default bench (all legs), then the limiter legs' profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_limiters.py tests/test_gpu_pipeline.py tests/test_gpu_heavy.py > gpurun_out/r04s_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/r04s_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/shard_kernels.py 8 > gpurun_out/r04s_shard_kernels.json 2>&1; echo shard_rc=$?; tail -c 700 gpurun_out/r04s_shard_kernels.json
timeout -k 10 600 python3 bench.py > gpurun_out/r04s_bench.log 2>&1
rc=$?; echo bench_rc=$rc; [ $rc -eq 0 ] || exit $rc
PROF_TAG=r04s bash scripts/gpu_r04_legs_prof.sh
