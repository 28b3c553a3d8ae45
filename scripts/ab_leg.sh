#!/bin/bash
# A/B of one bench leg under environment switches: scripts/ab_leg.sh LEG "ENV1" "ENV2" ...
# ("" = the defaults), e.g. scripts/ab_leg.sh config5 "" "FSX_CLEAR_MEMSET=1". Prints the
# leg's ms per step for each setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
leg=$1; shift
for e in "$@"; do
  env $e timeout -k 10 400 python bench.py --steps 3 --warmup 1 --packets 1048576 --no-cpu-baseline --no-check \
      --legs "$leg" --kernel-timing-steps 0 ${AB_ARGS:-} > gpurun_out/abl.json 2> gpurun_out/abl.err || exit $?
  python - "$leg" "$e" <<'PY'
import json, sys
leg, e = sys.argv[1], sys.argv[2]
d = json.loads(open("gpurun_out/abl.json").read().strip().splitlines()[-1])
r = d[{"rules": "prefix_rules"}.get(leg, leg)]
if "ms_per_step" in r:
    print(e or "default", leg, r["ms_per_step"])
else:   # (a leg of several runs: limiters)
    print(e or "default", leg, {k: v["ms_per_step"] for k, v in r.items() if isinstance(v, dict) and "ms_per_step" in v})
PY
done
