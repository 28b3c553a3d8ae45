#!/bin/bash
# A/B timing of library variants on the GPU box: scripts/ab.sh "" s3 s2 ...
# ("" = the product build). Prints ms/step and the per-kernel split of each.
# AB_MLP=0 drops features + scores from the step (default: the headline step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  FSX_LIB_VARIANT=$v timeout -k 10 240 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-check --legs "" $([ "${AB_MLP:-1}" = 1 ] || echo --no-mlp) ${AB_ARGS:-} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{v}.json").read().strip().splitlines()[-1])
print(v or "base", d["ms_per_step"], [(k["name"], k["ms_per_step"]) for k in d["kernels"]])
PY
done
