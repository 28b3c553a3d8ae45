#!/bin/bash
# A/B of run-time switches on the headline stream (pipelined) and its unpipelined twin:
#   scripts/ab_stream.sh "" "FSX_STREAM_PRIO=-1,0,0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for v in "$@"; do
  k=$((k + 1))
  env $v timeout -k 10 240 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --legs ${AB_LEGS:-unpipelined} \
      --no-check --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/abs_$k.json 2> gpurun_out/abs_$k.err || exit $?
  python - "$k" "$v" <<'PY'
import json, sys
k, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/abs_{k}.json").read().strip().splitlines()[-1])
print(v or "defaults", "stream pipelined", d["ms_per_step"], "unpipelined",
      (d.get("unpipelined") or {}).get("ms_per_step"), "cold", (d.get("cold") or {}).get("ms_per_step"),
      [(x["name"], x["ms_per_step"]) for x in d["kernels"]], flush=True)
PY
done
