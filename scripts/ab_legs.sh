#!/bin/bash
# A/B of run-time switches on the config-4 share and the config-5 carpet legs:
#   scripts/ab_legs.sh "" "FSX_NO_MIRROR=1"
# Prints one line per (variant, leg) with ms per step; logs in gpurun_out/abl_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for v in "$@"; do
  k=$((k + 1))
  env $v timeout -k 10 300 python bench.py --config 4 --packets 134217728 --steps ${AB_STEPS:-5} --warmup 2 \
      --legs "" --no-check --no-cpu-baseline > gpurun_out/abl_c4_$k.json 2> gpurun_out/abl_c4_$k.err || exit $?
  env $v timeout -k 10 300 python bench.py --packets 1048576 --steps 2 --warmup 1 --legs config5 \
      --no-config5-oracle --no-check --no-cpu-baseline --leg-steps ${AB_LEG_STEPS:-6} \
      > gpurun_out/abl_c5_$k.json 2> gpurun_out/abl_c5_$k.err || exit $?
  python - "$k" "$v" <<'PY'
import json, sys
k, v = sys.argv[1], sys.argv[2]
c4 = json.loads(open(f"gpurun_out/abl_c4_{k}.json").read().strip().splitlines()[-1])
c5 = json.loads(open(f"gpurun_out/abl_c5_{k}.json").read().strip().splitlines()[-1])
print(v or "defaults", "config4 ms/step", c4["ms_per_step"], "k_parse", c4["roofline"]["launch_ms"],
      "config5 ms/step", (c5.get("config5") or {}).get("ms_per_step"), flush=True)
PY
done
