#!/bin/bash
# Build the micro-benchmarks for gfx950 (in this container; the binaries travel).
set -e
cd "$(dirname "$0")"
for m in ${@:-stream_micro}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
    -I../../include -I../../flowsentryx_amd/csrc -o $m $m.hip
done
