#!/bin/bash
# A/B tuning build: libfsx_hip.<name>.so from the product sources with extra -D flags,
# selected at run time with FSX_LIB_VARIANT=<name> (flowsentryx_amd/lib.py).
#   scripts/build_variant.sh scat3 -DFSX_SCATTER_MINB=3
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
python3 - "$name" "$@" <<'PY'
import subprocess, sys
from flowsentryx_amd import build as b
name, defs = sys.argv[1], sys.argv[2:]
out = b.PKG / f"libfsx_hip.{name}.so"
cmd = [b.HIPCC, *b.COMMON, *defs, "-o", str(out), *[str(b.CSRC / s) for s in b.LIBS["libfsx_hip.so"]]]
r = subprocess.run(cmd, capture_output=True, text=True)
if r.returncode:
    sys.exit(r.stderr)
print(out)
PY
