# Kernel trace + stats and HBM PMC passes of the headline workload under the sliding
# window and the token bucket (bench.py --limiter), for the limiters' roofline evidence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lim in ${LIMS:-sliding token}; do
  PROF_TAG=${PROF_TAG:-r04k}_$lim BENCH_ARGS="--limiter $lim" bash scripts/gpu_profile.sh || exit $?
  PMC_MORE=0 PROF_TAG=${PROF_TAG:-r04k}_$lim BENCH_ARGS="--limiter $lim" bash scripts/gpu_pmc.sh || exit $?
done
