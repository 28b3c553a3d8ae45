"""Build recipe for the in-tree native libraries (gfx950 only).

libfsx_hip.so    the product: C-ABI of include/fsx_hip.h (hot-path kernels + host API)
libfsx_synth.so  synthetic packet streams on device (bench / tests)

Both are built with `hipcc --offload-arch=gfx950` straight into this package
directory, so they travel with the repo snapshot to the GPU box. The CPU oracle
(oracle/Makefile) is test infrastructure and is built by `build_oracle()`.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("FSX_OFFLOAD_ARCH", "gfx950")
COMMON = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-Wall", "-Wshadow", "-Wno-unused-function", "-Wno-unused-variable",
    f"-I{INCLUDE}", f"-I{CSRC}",
]

LIBS = {
    "libfsx_hip.so": ["fsx_device.hip", "fsx_limiters.hip", "fsx_shard.hip", "fsx_pcap.hip",
                      "fsx_flows.hip", "fsx_score.hip", "fsx_heavy.hip",
                      "fsx_api.hip"],
    "libfsx_synth.so": ["fsx_synth.hip"],
}
HEADERS = ["fsx_internal.h", "fsx_synth_common.h", "fsx_dev_common.h", "fsx_q8.h", "fsx_seg.h", "fsx_shard.h", "fsx_walk.h",
           "fsx_flow_common.h", "fsx_heavy_view.h", "fsx_search.h"]


def _stale(out: Path, srcs: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    deps = srcs + [CSRC / h for h in HEADERS] + [INCLUDE / "fsx_hip.h", Path(__file__)]
    return any(d.exists() and d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path, extra: list[str]) -> None:
    cmd = [HIPCC, *[f for f in COMMON if f != "-shared"], *extra, "-c", "-o", str(obj), str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")


def build_lib(name: str, force: bool = False, verbose: bool = False,
              only_missing: bool = False, extra: list[str] | None = None, out: Path | None = None) -> Path:
    """One translation unit per source, compiled in parallel (objects under build/), then
    linked into the shared library. `extra` / `out`: A/B variants (scripts/build_variant.sh)."""
    from concurrent.futures import ThreadPoolExecutor
    out = out or PKG / name
    srcs = [CSRC / s for s in LIBS[name]]
    if only_missing and out.exists() and not force:
        return out
    if not force and not extra and not _stale(out, srcs):
        return out
    objdir = ROOT / "build" / (out.name + ".obj")
    objdir.mkdir(parents=True, exist_ok=True)
    objs = [objdir / (s.stem + ".o") for s in srcs]
    if verbose:
        print(f"hipcc {len(srcs)} sources -> {out.name}", file=sys.stderr)
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda so: _compile(so[0], so[1], list(extra or [])), zip(srcs, objs)))
    tmp = out.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed for {name}:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = False, only_missing: bool = False) -> list[Path]:
    return [build_lib(n, force, verbose, only_missing) for n in LIBS]


def build_oracle(verbose: bool = False) -> None:
    """Test infrastructure: CPU oracle (+ oracle/_ref when the reference exists)."""
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "all"], capture_output=True, text=True)
    if verbose:
        print(r.stdout, r.stderr, file=sys.stderr)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(force=force, verbose=True):
        print(p)
    build_oracle(verbose=True)
