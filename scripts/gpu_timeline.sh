#!/bin/bash
# Kernel timeline of one bench step (rocprofv3 kernel trace, no counters): prints the
# last step's kernels with start / end offsets (us) and queue. Env is passed through
# (e.g. FSX_NO_FLOW_FORK=1 scripts/gpu_timeline.sh).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/tl_${TL_TAG:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-check --legs none --kernel-timing-steps 0 ${BENCH_ARGS:-} \
  > "$OUT/bench_stdout.log" 2>&1 || exit $?
python3 "$REPO/scripts/timeline.py" "$OUT/run_kernel_trace.csv"
