# A/B: split pipelining for the sliding window and the token bucket.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lim in token sliding; do
  AB_ARGS="--limiter $lim" AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_SPLIT_FIXED_ONLY=1" "" "FSX_SPLIT_FIXED_ONLY=1" > gpurun_out/ab_r04t_$lim.txt 2>&1 || exit $?
  echo $lim; cut -c1-70 gpurun_out/ab_r04t_$lim.txt
done
