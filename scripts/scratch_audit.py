#!/usr/bin/env python3
"""Per-kernel scratch (private segment) and register use of a built library.

Reads the gfx950 code object out of the library's clang offload bundle and its AMDGPU
metadata note (llvm-readelf --notes), so the audit covers exactly the code that ships.

    python3 scripts/scratch_audit.py [flowsentryx_amd/libfsx_hip.so] [--all]

Prints one line per kernel with scratch (or every kernel with --all)."""
from __future__ import annotations

import shutil
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parent.parent
READELF = shutil.which("llvm-readelf") or "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(lib: Path, arch: str = "gfx950") -> list[bytes]:
    """The arch's code object of every offload bundle (one per translation unit)."""
    data = lib.read_bytes()
    out = []
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    while i >= 0:
        off = i + 24
        (n,) = struct.unpack_from("<Q", data, off)
        off += 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if triple.endswith(arch):
                co = data[i + o:i + o + sz]
                if co[:4] != b"\x7fELF":
                    raise RuntimeError(f"{lib}: {triple} code object is not a plain ELF (compressed?)")
                out.append(co)
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 24)
    if not out:
        raise RuntimeError(f"{lib}: no {arch} code object")
    return out


def kernels(lib: Path) -> list[dict]:
    """[{name, scratch, vgpr, agpr, sgpr, lds}] of every kernel in the library."""
    out = []
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True,
                                 check=True).stdout
        a = txt.index("---")
        b = txt.index("\n...", a)
        meta = yaml.safe_load(txt[a:b])
        for k in meta.get("amdhsa.kernels", []):
            out.append({"name": k[".name"], "scratch": k[".private_segment_fixed_size"],
                        "vgpr": k[".vgpr_count"], "agpr": k.get(".agpr_count", 0),
                        "sgpr": k[".sgpr_count"], "lds": k[".group_segment_fixed_size"]})
    return out


def main() -> None:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = Path(args[0]) if args else ROOT / "flowsentryx_amd" / "libfsx_hip.so"
    for k in sorted(kernels(lib), key=lambda k: (-k["scratch"], k["name"])):
        if k["scratch"] or "--all" in sys.argv:
            print(f"{k['scratch']:5d} B scratch  {k['vgpr']:4d} vgpr  {k['lds']:6d} B lds  {k['name']}")


if __name__ == "__main__":
    main()
