"""CPU: the C ABI library loads and exports every symbol include/fsx_hip.h declares;
host-side logic that needs no GPU (config defaults, error paths, struct layouts)."""
import ctypes as C
import errno
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "fsx_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fsx_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree(native):
    assert declared_symbols() == sorted(native.ABI_SYMBOLS)


def test_library_exports_all_symbols(native):
    lib = native.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.fsx_abi_version() == 1


def test_config_defaults_are_reference_constants(native):
    cfg = native.default_config()
    assert cfg.pps_threshold == 1000          # src/fsx_kern.c:309
    assert cfg.bps_threshold == 125_000_000   # src/fsx_kern.c:310
    assert cfg.window_ns == 1_000_000_000     # src/fsx_kern.c:245
    assert cfg.block_ns == 10_000_000_000     # src/fsx_kern.c:308,317
    assert cfg.max_entries == 100_000         # src/fsx_struct.h:7
    assert cfg.limiter == native.LIMIT_FIXED_WINDOW


def test_struct_layouts(native):
    assert C.sizeof(native.FsxStats) == 16      # struct stats, src/fsx_struct.h:11-15
    assert C.sizeof(native.FsxConfig) == 9 * 8 + 3 * 4 + 7 * 4
    assert C.sizeof(native.FsxQ8Model) == 8 + 6 * 4


def test_reference_struct_sizes_match(oracle):
    """The reference's own fsx_struct.h, compiled into oracle/_ref, agrees on layouts."""
    if not oracle.REF_LIB.exists():
        pytest.skip("oracle/_ref not built")
    L = C.CDLL(str(oracle.REF_LIB))
    L.ref_sizeof_stats.restype = C.c_size_t
    L.ref_sizeof_ip_stats.restype = C.c_size_t
    assert L.ref_sizeof_stats() == 16 and L.ref_sizeof_ip_stats() == 24


def test_open_without_gpu_fails_loudly(native):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(native.FsxError) as e:
        native.FsxContext()
    assert e.value.code in (-errno.ENODEV, -errno.EINVAL, -errno.EIO)


def test_bad_config_rejected(native):
    lib = native.load_library()
    h = C.c_void_p()
    cfg = native.default_config(max_entries=0)
    assert lib.fsx_open(C.byref(h), C.byref(cfg)) == -errno.EINVAL
    cfg = native.default_config(limiter=7)
    assert lib.fsx_open(C.byref(h), C.byref(cfg)) == -errno.EINVAL
    assert lib.fsx_open(None, None) == -errno.EINVAL
