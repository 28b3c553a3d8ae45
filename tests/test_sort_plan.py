"""CPU: the radix sort's digit plan (flowsentryx_amd/csrc/fsx_plan.h), the host function
launch_verdict_pipeline uses to pick a batch's passes and digit ranges. Compiled with g++ into a
harness (tests/csrc/sort_plan.cpp) that walks every id width 1..32 under every combination of
the plan's switches and checks what the kernels assume: at most 9-bit digits (512-digit tiles),
8-bit ones wherever k_parse counts them, id bits tiled exactly and contiguously, the heavy
bucket above the id, an even pass count only with the fixed window's heavy lists, tile-scan
bases exactly for the 9-bit plans; plus the plans of the BASELINE tables."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_sort_plan_invariants(tmp_path):
    exe = tmp_path / "sort_plan"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", f"-I{ROOT / 'flowsentryx_amd' / 'csrc'}",
                    str(ROOT / "tests" / "csrc" / "sort_plan.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
