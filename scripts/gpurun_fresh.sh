#!/bin/bash
# Local helper: rebuild stale in-tree libraries, then run a command on the GPU box.
# usage: scripts/gpurun_fresh.sh <timeout-s> '<command>'
set -e
cd "$(dirname "$0")/.."
python -c "from flowsentryx_amd import build; build.build_all()"
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
