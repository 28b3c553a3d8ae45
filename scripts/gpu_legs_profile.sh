#!/bin/bash
# rocprofv3 kernel-trace + stats of ONE bench leg run as the headline (so the summary holds
# that workload's kernels only): LEG=config4 (one rank's 1/8 share of the 1B-packet stream),
# LEG=config3 (the 4M-flow stream), LEG=config2 (the headline), LEG=config5 (the 2^28-packet
# carpet leg beside a 1M-packet headline: its block in the line, its kernels in the stats). Output:
# gpurun_out/prof_${PROF_TAG}/ (kernel_stats.csv + the bench line).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
LEG="${LEG:-config4}"
OUT="$REPO/gpurun_out/prof_${PROF_TAG:-r03_$LEG}"
mkdir -p "$OUT"
case "$LEG" in
  config4) ARGS="--config 4 --packets 134217728" ;;
  config3) ARGS="--config 3" ;;
  config5) ARGS="--packets 1048576 --legs config5 --no-config5-oracle" ;;
  *) ARGS="" ;;
esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps ${PROF_STEPS:-4} --warmup 1 --no-cpu-baseline --no-check --legs "" $ARGS \
  ${BENCH_ARGS:-} > "$OUT/bench_under_rocprof.log" 2>&1
rc=$?
echo "profile $LEG rc=$rc"
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
exit $rc
