# Sharded local kernels at G = 8 (pack + warm owner record batches), then the limiter legs'
# kernel traces + HBM PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/shard_kernels.py 8 > gpurun_out/r04o_shard_kernels.json 2>&1
rc=$?; echo shard_rc=$rc; tail -c 800 gpurun_out/r04o_shard_kernels.json; [ $rc -eq 0 ] || exit $rc
PROF_TAG=r04o bash scripts/gpu_r04_legs_prof.sh
