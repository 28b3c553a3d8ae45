# With the tail before the parse: the token bucket split (FSX_SPLIT_TOKEN=1) against whole,
# the sliding window whole (FSX_SPLIT_FIXED_ONLY=1) against split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_ARGS="--limiter token" AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_SPLIT_TOKEN=1" "" "FSX_SPLIT_TOKEN=1" > gpurun_out/ab_r04ad_token.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04ad_token.txt
AB_ARGS="--limiter sliding" AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_SPLIT_FIXED_ONLY=1" "" "FSX_SPLIT_FIXED_ONLY=1" > gpurun_out/ab_r04ad_sliding.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04ad_sliding.txt
