"""The shipped code object keeps its kernels in registers: no scratch (private segment)
in any product kernel except the sort scatter's measured late-payload variant, whose
24 B/lane of spills at 4 waves / SIMD (three tile slots and one address, once per tile)
won the occupancy A/B. Read from the built library's own metadata."""
import shutil
from pathlib import Path

import pytest

from scripts import scratch_audit

ALLOWED = {"_ZN3fsx14k_tile_scatterILb1EEEvPKmPmjPKjjjiS5_jPKNS_10BatchStateES2_S3_S2_S5_": 24}


@pytest.fixture(scope="module")
def kernels(native):
    if not Path(scratch_audit.READELF).exists() and not shutil.which("llvm-readelf"):
        pytest.skip("llvm-readelf not available")
    return scratch_audit.kernels(Path(native.__file__).parent / "libfsx_hip.so")


def test_no_unexpected_scratch(kernels):
    bad = {k["name"]: k["scratch"] for k in kernels
           if k["scratch"] and ALLOWED.get(k["name"], 0) < k["scratch"]}
    assert not bad, bad


def test_flow_and_walker_kernels_scratch_free(kernels):
    names = [k for k in kernels if any(s in k["name"] for s in ("k_flow", "k_walk", "k_tb_", "k_sw_"))]
    assert len(names) >= 10
    assert all(k["scratch"] == 0 for k in names), [k["name"] for k in names if k["scratch"]]
