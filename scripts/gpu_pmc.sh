#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only, no runtime/sys traces) of a
# short bench run: HBM-side FETCH_SIZE and WRITE_SIZE per dispatch, then SQ counters.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${PROF_TAG:-r01}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$tag" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "pmc $tag rc=$rc"
  return $rc
}
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
find "$OUT" -name "*counter_collection*"
