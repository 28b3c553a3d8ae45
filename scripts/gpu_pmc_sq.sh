#!/bin/bash
# SQ counter passes only (instruction mix, waits, LDS bank conflicts) of a short headline run.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${PROF_TAG:-sq}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$tag" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-check --legs "" ${BENCH_ARGS:-} \
    > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "pmc $tag rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit $?
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA || exit $?
