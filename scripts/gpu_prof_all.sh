#!/bin/bash
# One GPU session of evidence: kernel-trace stats of a short bench, then the PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
