#!/bin/bash
# A/B on one box: the headline with the heavy sources outside the sort (default) against the
# run path (FSX_NO_HFAST=1), interleaved, then a kernel trace of the default.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/ab_hfast_${AB_TAG:-r04}"
mkdir -p "$OUT"
cd "$REPO"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --legs "" --no-cpu-baseline --no-check \
    > "$OUT/hfast_$i.log" 2>&1 || exit $?
  FSX_NO_HFAST=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --legs "" --no-cpu-baseline --no-check \
    > "$OUT/runs_$i.log" 2>&1 || exit $?
done
for f in "$OUT"/*.log; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'])" "$f"
done
