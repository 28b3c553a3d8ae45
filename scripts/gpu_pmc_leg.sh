#!/bin/bash
# HBM bytes per batch of one bench leg: FETCH_SIZE and WRITE_SIZE passes (kernel-trace only)
# of a bench run with only that leg (the headline shrunk to 1M packets), then
# scripts/leg_pmc.py.   PROF_TAG=... LEG=config5 bash scripts/gpu_pmc_leg.sh
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${PROF_TAG:-leg}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 500 rocprofv3 --kernel-trace --pmc "$c" --output-format csv -d "$OUT/$c" -o run -- \
    python3 "$REPO/bench.py" --steps 1 --warmup 1 --packets 1048576 --no-cpu-baseline --no-check \
    --legs "${LEG:-config5}" --leg-steps 2 --kernel-timing-steps 0 > "$OUT/$c.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 "$REPO/scripts/leg_pmc.py" "$OUT" > "$OUT/per_batch.txt" && cat "$OUT/per_batch.txt"
