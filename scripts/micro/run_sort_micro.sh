#!/bin/bash
# GPU box: run the prebuilt sort micro-benchmark (built here by build_micro.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/sort_micro "$@" > gpurun_out/sort_micro.log 2>&1
rc=$?
cat gpurun_out/sort_micro.log
exit $rc
