# Tuning A/B after the round-4 changes: flow-tile grid, short-walker grid, short-segment
# bound, sort-scatter occupancy (headline, then config 4 for the flow-tile grid).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh "" ftb1k wsb1k ss128 scat3 "" ftb1k scat3 > gpurun_out/ab_r04z.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04z.txt
for v in "" ftb1k "" ftb1k; do
  FSX_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --legs config4 --leg-steps 4 --no-check \
    --no-cpu-baseline > gpurun_out/r04z_c4_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r04z_c4_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1] or "cur", "config4", d["config4"]["ms_per_step"])
PY
done
