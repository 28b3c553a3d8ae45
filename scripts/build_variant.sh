#!/bin/bash
# A/B tuning build: libfsx_hip.<name>.so from the product sources with extra -D flags,
# selected at run time with FSX_LIB_VARIANT=<name> (flowsentryx_amd/lib.py).
#   scripts/build_variant.sh scat3 -DFSX_SCATTER_MINB=3
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
python3 - "$name" "$@" <<'PY'
import sys
from flowsentryx_amd import build as b
name, defs = sys.argv[1], sys.argv[2:]
print(b.build_lib("libfsx_hip.so", extra=defs, out=b.PKG / f"libfsx_hip.{name}.so"))
PY
