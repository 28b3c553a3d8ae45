#!/bin/bash
# HBM traffic of the sharded path's local kernels (scripts/shard_kernels.py, G = 8): one
# counter per pass (FETCH_SIZE, WRITE_SIZE), kernel-trace only.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${PROF_TAG:-shard}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc "$c" --output-format csv -d "$OUT/$c" -o run -- \
    python3 "$REPO/scripts/shard_kernels.py" 8 > "$OUT/$c.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name "*counter_collection*"
