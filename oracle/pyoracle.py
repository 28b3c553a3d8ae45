"""ctypes binding of the CPU oracle (oracle/build/libfsx_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker. The product (flowsentryx_amd/) never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libfsx_oracle.so"
REF_LIB = HERE / "_ref" / "libref_parse.so"


class OConfig(C.Structure):
    _fields_ = [
        ("pps_threshold", C.c_uint64), ("bps_threshold", C.c_uint64),
        ("window_ns", C.c_uint64), ("block_ns", C.c_uint64), ("max_entries", C.c_uint64),
        ("tb_rate", C.c_uint64), ("tb_burst", C.c_uint64),
        ("limiter", C.c_int32), ("flags", C.c_int32),
    ]


EVICT_IDLE = 4   # fsxo_config.flags, = include/fsx_hip.h FSX_FLAG_EVICT_IDLE
OVERFLOW_ADMIT = 8   # = include/fsx_hip.h FSX_FLAG_OVERFLOW_ADMIT


class OQ8Model(C.Structure):
    _fields_ = [
        ("weight", C.c_int8 * 8), ("weight_scale", C.c_float), ("bias", C.c_float),
        ("in_scale", C.c_float), ("in_zero_point", C.c_int32), ("out_scale", C.c_float),
        ("out_zero_point", C.c_int32),
    ]


_lib = None


def build():
    r = subprocess.run(["make", "-C", str(HERE), "build/libfsx_oracle.so"], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stdout + r.stderr)


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        build()
    L = C.CDLL(str(LIB))
    vp, sz = C.c_void_p, C.c_size_t
    sig = {
        "fsxo_config_default": (None, [C.POINTER(OConfig)]),
        "fsxo_open": (vp, [C.POINTER(OConfig)]),
        "fsxo_close": (None, [vp]),
        "fsxo_reset": (None, [vp]),
        "fsxo_error": (C.c_int, [vp]),
        "fsxo_get_stats": (None, [vp, vp]),
        "fsxo_batch": (C.c_int, [vp, vp, vp, vp, sz, vp]),
        "fsxo_evicted_last": (C.c_uint64, [vp]),
        "fsxo_admit_last": (None, [vp, vp]),
        "fsxo_parse_batch": (None, [vp, vp, sz, vp, vp]),
        "fsxo_map_lookup": (C.c_int, [vp, C.c_int, vp, vp]),
        "fsxo_map_update": (C.c_int, [vp, C.c_int, vp, vp]),
        "fsxo_map_delete": (C.c_int, [vp, C.c_int, vp]),
        "fsxo_map_dump": (sz, [vp, C.c_int, vp, vp, sz]),
        "fsxo_batch_sharded": (C.c_int, [C.POINTER(OConfig), vp, vp, vp, sz, vp, C.c_int, vp]),
        "fsxo_shards_open": (vp, [C.POINTER(OConfig), C.c_int]),
        "fsxo_shards_close": (None, [vp]),
        "fsxo_shards_reset": (None, [vp]),
        "fsxo_shards_map_update": (C.c_int, [vp, C.c_int, vp, vp]),
        "fsxo_shards_batch": (C.c_int, [vp, vp, vp, vp, sz, vp]),
        "fsxo_shards_stats": (None, [vp, vp]),
        "fsxo_shards_dump": (sz, [vp, C.c_int, vp, vp, sz]),
        "fsxo_sigmoid_lut": (None, [C.c_float, C.c_int32, vp]),
        "fsxo_score": (None, [C.POINTER(OQ8Model), vp, sz, vp, vp, vp]),
        "fsxo_flow_features": (sz, [vp, vp, vp, sz, sz, vp, vp, vp, sz]),
        "fsxo_synth": (C.c_int, [vp, C.c_double, C.c_uint64, sz, vp, vp, vp]),
        "fsxo_zipf_alias": (C.c_int, [C.c_uint32, C.c_double, vp, vp]),
        "fsxo_dst_port": (C.c_uint32, [vp, C.c_uint32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def default_config(**kw) -> OConfig:
    c = OConfig()
    lib().fsxo_config_default(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


class Oracle:
    """Sequential restatement of fsx() + its maps (src/fsx_kern.c:56-347)."""

    def __init__(self, **kw):
        self.cfg = default_config(**kw)
        self._h = lib().fsxo_open(C.byref(self.cfg))
        if not self._h:
            raise MemoryError("fsxo_open")

    def close(self):
        if self._h:
            lib().fsxo_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def batch(self, hdr, length, ts) -> np.ndarray:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        out = np.empty(hdr.shape[0], dtype=np.uint8)
        rc = lib().fsxo_batch(self._h, _p(hdr), _p(length), _p(ts), hdr.shape[0], _p(out))
        if rc:
            raise RuntimeError(f"oracle error {rc}")
        return out

    def stats(self) -> tuple[int, int]:
        s = np.zeros(2, dtype=np.uint64)
        lib().fsxo_get_stats(self._h, _p(s))
        return int(s[0]), int(s[1])

    def evicted_last(self) -> int:
        """Sources evicted before the last batch (flags=EVICT_IDLE)."""
        return int(lib().fsxo_evicted_last(self._h))

    def admit_last(self) -> tuple[int, int]:
        """Sources admitted / transient in the last batch (flags=OVERFLOW_ADMIT)."""
        s = np.zeros(2, dtype=np.uint64)
        lib().fsxo_admit_last(self._h, _p(s))
        return int(s[0]), int(s[1])

    def reset(self):
        """fsx_reset's counterpart: per-source maps and stats cleared, prefix rules kept."""
        lib().fsxo_reset(self._h)

    def map_update(self, map_id: int, key: bytes, value):
        if map_id in (1, 2, 5, 6):
            v = np.array(value, dtype=np.uint64)
        else:
            v = np.array([value], dtype=np.uint64)
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        rc = lib().fsxo_map_update(self._h, map_id, _p(k), _p(v))
        if rc:
            raise RuntimeError(f"oracle map update {rc}")

    def map_lookup(self, map_id: int, key: bytes):
        """Scalar value (blacklists, prefix maps: longest match) or None."""
        vw = 3 if map_id in (1, 2) else 2 if map_id in (5, 6) else 1
        v = np.zeros(vw, dtype=np.uint64)
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        rc = lib().fsxo_map_lookup(self._h, map_id, _p(k), _p(v))
        if rc:
            return None
        return tuple(int(x) for x in v) if vw > 1 else int(v[0])

    def map_delete(self, map_id: int, key: bytes) -> int:
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        return lib().fsxo_map_delete(self._h, map_id, _p(k))

    def map_dump(self, map_id: int) -> dict:
        klen = 16 if map_id in (2, 4, 6) else 8 if map_id == 7 else 20 if map_id == 8 else 4
        vw = 3 if map_id in (1, 2) else 2 if map_id in (5, 6) else 1
        n = lib().fsxo_map_dump(self._h, map_id, None, None, 0)
        keys = np.zeros((max(n, 1), klen), dtype=np.uint8)
        vals = np.zeros((max(n, 1), vw), dtype=np.uint64)
        lib().fsxo_map_dump(self._h, map_id, _p(keys), _p(vals), n)
        return {keys[i].tobytes(): (tuple(int(x) for x in vals[i]) if vw > 1 else int(vals[i, 0]))
                for i in range(n)}

    def map_arrays(self, map_id: int):
        """(keys [n, klen] u8, values [n, words] u64) of one map, unordered."""
        n = lib().fsxo_map_dump(self._h, map_id, None, None, 0)
        keys = np.zeros((n, _klen(map_id)), dtype=np.uint8)
        vals = np.zeros((n, _vw(map_id)), dtype=np.uint64)
        if n:
            lib().fsxo_map_dump(self._h, map_id, _p(keys), _p(vals), n)
        return keys, vals


def _klen(map_id: int) -> int:
    return 16 if map_id in (2, 4, 6) else 8 if map_id == 7 else 20 if map_id == 8 else 4


def _vw(map_id: int) -> int:
    return 3 if map_id in (1, 2) else 2 if map_id in (5, 6) else 1


def _map_value(map_id: int, value) -> np.ndarray:
    return np.array(value if map_id in (1, 2, 5, 6) else [value], dtype=np.uint64)


class ShardedOracle:
    """The sequential oracle on T host threads over IP-disjoint shards, with persistent
    maps (fsxo_shards_*): verdicts, stats_map and map dumps equal one Oracle's for the
    same stream (per-source arrival order is kept), in 1/T of the time. Used for the
    full-size checks (bench.py, large GPU tests); -ENOSPC is not reproduced."""

    def __init__(self, nthreads: int, **kw):
        self.cfg = default_config(**kw)
        self._h = lib().fsxo_shards_open(C.byref(self.cfg), int(nthreads))
        if not self._h:
            raise MemoryError("fsxo_shards_open")

    def close(self):
        if self._h:
            lib().fsxo_shards_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def reset(self):
        lib().fsxo_shards_reset(self._h)

    def batch(self, hdr, length, ts) -> np.ndarray:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        out = np.empty(hdr.shape[0], dtype=np.uint8)
        rc = lib().fsxo_shards_batch(self._h, _p(hdr), _p(length), _p(ts), hdr.shape[0], _p(out))
        if rc:
            raise RuntimeError(f"oracle error {rc}")
        return out

    def stats(self) -> tuple[int, int]:
        s = np.zeros(2, dtype=np.uint64)
        lib().fsxo_shards_stats(self._h, _p(s))
        return int(s[0]), int(s[1])

    def map_update(self, map_id: int, key: bytes, value):
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        v = _map_value(map_id, value)
        rc = lib().fsxo_shards_map_update(self._h, map_id, _p(k), _p(v))
        if rc:
            raise RuntimeError(f"oracle map update {rc}")

    def map_arrays(self, map_id: int):
        """(keys [n, klen] u8, values [n, words] u64) of one map, unordered."""
        n = lib().fsxo_shards_dump(self._h, map_id, None, None, 0)
        keys = np.zeros((n, _klen(map_id)), dtype=np.uint8)
        vals = np.zeros((n, _vw(map_id)), dtype=np.uint64)
        if n:
            lib().fsxo_shards_dump(self._h, map_id, _p(keys), _p(vals), n)
        return keys, vals


def sort_map_arrays(keys: np.ndarray, vals: np.ndarray):
    """Rows of a map dump in key order (any key width), for array comparisons."""
    k = np.ascontiguousarray(keys, dtype=np.uint8)
    if k.shape[0] == 0:
        return k, vals
    w = (k.shape[1] + 7) // 8 * 8
    kp = np.zeros((k.shape[0], w), dtype=np.uint8)
    kp[:, :k.shape[1]] = k
    cols = kp.view(">u8")   # big-endian words: byte-lexicographic order
    order = np.lexsort(cols.T[::-1])
    return k[order], np.ascontiguousarray(vals)[order]


def same_map(a, b) -> bool:
    """Two (keys, values) dumps hold the same entries."""
    ka, va = sort_map_arrays(*a)
    kb, vb = sort_map_arrays(*b)
    return ka.shape == kb.shape and np.array_equal(ka, kb) and np.array_equal(va, vb)


def parse(hdr, length):
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    n = hdr.shape[0]
    cls = np.zeros(n, dtype=np.uint8)
    keys = np.zeros((n, 16), dtype=np.uint8)
    lib().fsxo_parse_batch(_p(hdr), _p(length), n, _p(cls), _p(keys))
    return cls, keys


def ref_parse(hdr, length):
    """The reference's own parsing_helper.h (oracle/_ref), when it was built here."""
    if not REF_LIB.exists():
        raise FileNotFoundError(REF_LIB)
    L = C.CDLL(str(REF_LIB))
    L.ref_parse_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    n = hdr.shape[0]
    cls = np.zeros(n, dtype=np.uint8)
    keys = np.zeros((n, 16), dtype=np.uint8)
    L.ref_parse_batch(_p(hdr), _p(length), n, _p(cls), _p(keys))
    return cls, keys


def batch_sharded(hdr, length, ts, nthreads: int, **kw):
    cfg = default_config(**kw)
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    out = np.empty(hdr.shape[0], dtype=np.uint8)
    st = np.zeros(2, dtype=np.uint64)
    rc = lib().fsxo_batch_sharded(C.byref(cfg), _p(hdr), _p(length), _p(ts), hdr.shape[0],
                                  _p(out), nthreads, _p(st))
    if rc:
        raise RuntimeError(f"oracle error {rc}")
    return out, (int(st[0]), int(st[1]))


def q8_model(d: dict) -> OQ8Model:
    m = OQ8Model()
    for i, w in enumerate(d["weight"]):
        m.weight[i] = int(w)
    m.weight_scale = d["weight_scale"]
    m.bias = d["bias"]
    m.in_scale = d["in_scale"]
    m.in_zero_point = d["in_zero_point"]
    m.out_scale = d["out_scale"]
    m.out_zero_point = d["out_zero_point"]
    return m


def score(model: dict, feat):
    f = np.ascontiguousarray(feat, dtype=np.float32).reshape(-1, 8)
    n = f.shape[0]
    p = np.zeros(n, dtype=np.float32)
    d = np.zeros(n, dtype=np.uint8)
    lq = np.zeros(n, dtype=np.uint8)
    m = q8_model(model)
    lib().fsxo_score(C.byref(m), _p(f), n, _p(p), _p(d), _p(lq))
    return p, d, lq


def sigmoid_lut(out_scale: float, out_zp: int) -> np.ndarray:
    lut = np.zeros(256, dtype=np.uint8)
    lib().fsxo_sigmoid_lut(out_scale, out_zp, _p(lut))
    return lut


def flow_features(hdr, length, ts, max_sources: int | None = None):
    """Per-source features, sources in order of first appearance;
    max_sources (default n) sizes the tables (more sources raise)."""
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    n = hdr.shape[0]
    cap = max(1, min(n, max_sources or n))
    keys = np.zeros((cap, 16), dtype=np.uint8)
    fam = np.zeros(cap, dtype=np.uint8)
    feat = np.zeros((cap, 8), dtype=np.float32)
    nf = lib().fsxo_flow_features(_p(hdr), _p(length), _p(ts), n, cap, _p(keys), _p(fam),
                                  _p(feat), max_sources or 0)
    if nf == 2**64 - 1:
        raise ValueError(f"more than {max_sources} sources")
    return keys[:nf], fam[:nf], feat[:nf]


def synth(params, zipf_s: float, j0: int, count: int):
    """CPU twin of the device generator (flowsentryx_amd.synth.SynthParams)."""
    hdr = np.zeros((count, 64), dtype=np.uint8)
    length = np.zeros(count, dtype=np.uint32)
    ts = np.zeros(count, dtype=np.uint64)
    rc = lib().fsxo_synth(C.byref(params), zipf_s, j0, count, _p(hdr), _p(length), _p(ts))
    if rc:
        raise RuntimeError(f"fsxo_synth {rc}")
    return hdr, length, ts


def dst_port(hdr, length) -> np.ndarray:
    """L4 destination port per record (DESIGN.md §5 rule; 0 when absent)."""
    hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, 64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    f = lib().fsxo_dst_port
    return np.array([f(_p(hdr[i]), int(length[i])) for i in range(hdr.shape[0])], dtype=np.uint32)
