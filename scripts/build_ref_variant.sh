#!/bin/bash
# A/B against a committed version: libfsx_hip.<name>.so built from the csrc/ and include/
# of git ref <ref> (scripts/build_ref_variant.sh head HEAD), selected with FSX_LIB_VARIANT.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; ref=$2
tmp=$(mktemp -d)
cs="$tmp/flowsentryx_amd/csrc"
mkdir -p "$cs" "$tmp/include"
for f in $(git ls-tree --name-only "$ref" flowsentryx_amd/csrc/); do git show "$ref:$f" > "$cs/$(basename "$f")"; done
git show "$ref:include/fsx_hip.h" > "$tmp/include/fsx_hip.h"
srcs=""
for s in fsx_device.hip fsx_limiters.hip fsx_shard.hip fsx_pcap.hip fsx_flows.hip fsx_score.hip fsx_api.hip; do srcs="$srcs $cs/$s"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -w \
  -I"$tmp/include" -I"$cs" -o "flowsentryx_amd/libfsx_hip.$name.so" $srcs
rm -rf "$tmp"
echo "flowsentryx_amd/libfsx_hip.$name.so"
