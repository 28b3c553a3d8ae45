#!/bin/bash
# A/B timing of run-time switches on the GPU box: scripts/ab_env.sh "" "FSX_NO_HEAVY_LISTS=1" ...
# ("" = defaults). Each entry is a space-separated list of VAR=value settings for one run;
# prints ms/step and the per-kernel split (headline workload, no legs / checks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=0
for v in "$@"; do
  k=$((k + 1))
  env $v timeout -k 10 240 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --legs "" --no-check \
      --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/abenv_$k.json 2> gpurun_out/abenv_$k.err || exit $?
  python - "$k" "$v" <<'PY'
import json, sys
k, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/abenv_{k}.json").read().strip().splitlines()[-1])
print(v or "defaults", d["ms_per_step"], [(x["name"], x["ms_per_step"]) for x in d["kernels"]], flush=True)
PY
done
