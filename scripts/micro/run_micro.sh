#!/bin/bash
# GPU box: run one prebuilt micro-benchmark (built here by build_micro.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
m=$1; shift
timeout -k 10 120 ./scripts/micro/$m "$@" > gpurun_out/$m.log 2>&1
rc=$?
cat gpurun_out/$m.log
exit $rc
