#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this pass).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof_${PROF_TAG:-r01}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps ${PROF_STEPS:-5} --warmup 1 --no-cpu-baseline --legs "${PROF_LEGS:-}" ${BENCH_ARGS:-} \
  > "$OUT/bench_stdout.log" 2>&1
rc=$?
echo "profile rc=$rc"
find "$OUT" -name "*stats*" | head
exit $rc
