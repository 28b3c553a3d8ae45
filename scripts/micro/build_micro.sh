#!/bin/bash
# Build the micro-benchmarks for gfx950 (in this container; the binaries travel).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -I../../include -I../../flowsentryx_amd/csrc -o sort_micro sort_micro.hip
