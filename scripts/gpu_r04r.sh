# Warm owner batches in pipeline mode 0 / 2, then the headline A/B of the gated head loads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/dbg_owner_warm.py 2 > gpurun_out/r04r_owner_mode2.log 2>&1; echo mode2_rc=$?; grep " ms " gpurun_out/r04r_owner_mode2.log | cut -c1-40
AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_EAGER_SLOTS=1" "" "FSX_EAGER_SLOTS=1" > gpurun_out/ab_r04r.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04r.txt
