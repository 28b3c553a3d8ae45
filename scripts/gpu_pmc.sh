#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only, no runtime/sys traces) of a
# short bench run: HBM-side FETCH_SIZE and WRITE_SIZE per dispatch, SQ counters, L2 hits.
# BENCH_ARGS extends the bench command (default: headline only, no legs or checks).
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_${PROF_TAG:-r02}"
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
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit $?
if [ "${PMC_MORE:-1}" = 1 ]; then
  run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA || exit $?
  run tcc TCC_HIT_sum TCC_MISS_sum || exit $?
fi
find "$OUT" -name "*counter_collection*"
