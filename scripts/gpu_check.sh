#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Every GPU step has its own time
# limit; a crash/timeout/abort stops the script (test *failures* do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=240 --timeout-method=thread
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:-} || exit $?
