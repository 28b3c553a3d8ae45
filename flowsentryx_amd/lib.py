"""ctypes binding of libfsx_hip.so (include/fsx_hip.h).

This is the Python side of the drop-in boundary: the role src/fsx_load.py plays for
the reference (load the data plane, push model weights into it, read its maps),
calling the C ABI directly. It never falls back to a CPU path: if the native
library is missing or no GPU is present, opening a context raises FsxError.
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent

XDP_DROP = 1
XDP_PASS = 2
HDR_BYTES = 64

# enum fsx_map_id — the five maps of src/fsx_kern.c:56-94
MAP_STATS = 0
MAP_IPV4_STATS = 1
MAP_IPV6_STATS = 2
MAP_IPV4_BLACKLIST = 3
MAP_IPV6_BLACKLIST = 4
MAP_IPV4_TOKENS = 5   # build-defined token-bucket state
MAP_IPV6_TOKENS = 6
MAP_IPV4_PREFIX = 7   # build-defined prefix blocklists: LPM-trie keys
MAP_IPV6_PREFIX = 8
PREFIX_MAX_ENTRIES = 65536
MAP_NAMES = {
    MAP_STATS: "stats_map",
    MAP_IPV4_STATS: "ipv4_stats_map",
    MAP_IPV6_STATS: "ipv6_stats_map",
    MAP_IPV4_BLACKLIST: "ipv4_blacklist_map",
    MAP_IPV6_BLACKLIST: "ipv6_blacklist_map",
    MAP_IPV4_TOKENS: "ipv4_tokens_map",
    MAP_IPV6_TOKENS: "ipv6_tokens_map",
    MAP_IPV4_PREFIX: "ipv4_prefix_blocklist",
    MAP_IPV6_PREFIX: "ipv6_prefix_blocklist",
}
BPF_ANY, BPF_NOEXIST, BPF_EXIST = 0, 1, 2

# fsx_config.flags
FLAG_TEST_V6_COLLIDE = 1
FLAG_ONESWEEP_SORT = 2
FLAG_EVICT_IDLE = 4   # opt-in idle eviction on overflow
FLAG_OVERFLOW_ADMIT = 8   # opt-in admission of a flood's new sources
FLAG_SW_UNSORTED = 16     # A/B hook: the sliding window's heavy sources outside the sort
FLAG_TEST_SW_SPARSE = 32  # test hook: sparse heavy sources on the sliding window's run path
FLAG_ORDERED_INSERTS = 64  # home-ordered inserts on every fixed-window batch

LIMIT_FIXED_WINDOW = 0
LIMIT_SLIDING_WINDOW = 1
LIMIT_TOKEN_BUCKET = 2


class FsxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{errno.errorcode.get(-code, code)}] {msg}")
        self.code = code


class FsxConfig(C.Structure):
    _fields_ = [
        ("pps_threshold", C.c_uint64),
        ("bps_threshold", C.c_uint64),
        ("window_ns", C.c_uint64),
        ("block_ns", C.c_uint64),
        ("max_entries", C.c_uint64),
        ("max_batch", C.c_uint64),
        ("tb_rate", C.c_uint64),
        ("tb_burst", C.c_uint64),
        ("hash_seed", C.c_uint64),
        ("limiter", C.c_int32),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32 * 7),
    ]


class FsxStats(C.Structure):
    _fields_ = [("allowed", C.c_uint64), ("dropped", C.c_uint64)]


class FsxQ8Model(C.Structure):
    _fields_ = [
        ("weight", C.c_int8 * 8),
        ("weight_scale", C.c_float),
        ("bias", C.c_float),
        ("in_scale", C.c_float),
        ("in_zero_point", C.c_int32),
        ("out_scale", C.c_float),
        ("out_zero_point", C.c_int32),
    ]


_lib = None


def library_path() -> Path:
    # FSX_LIB_VARIANT=x loads libfsx_hip.x.so: in-tree A/B builds of the same sources
    # with different tuning macros (scripts/build_variant.sh); unset in production
    v = os.environ.get("FSX_LIB_VARIANT")
    return _PKG / (f"libfsx_hip.{v}.so" if v else "libfsx_hip.so")


def load_library() -> C.CDLL:
    """Load the in-tree libfsx_hip.so (fails loudly when it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not path.exists():
        raise FsxError(-errno.ENOENT,
                       f"{path} is not built: run `python -m flowsentryx_amd.build`")
    lib = C.CDLL(str(path))
    vp, sz, u8p = C.c_void_p, C.c_size_t, C.c_void_p
    sig = {
        "fsx_abi_version": (C.c_int, []),
        "fsx_config_default": (None, [C.POINTER(FsxConfig)]),
        "fsx_open": (C.c_int, [C.POINTER(vp), C.POINTER(FsxConfig)]),
        "fsx_close": (None, [vp]),
        "fsx_last_error": (C.c_char_p, [vp]),
        "fsx_set_stream": (C.c_int, [vp, vp]),
        "fsx_sync": (C.c_int, [vp]),
        "fsx_set_pipeline": (C.c_int, [vp, C.c_int]),
        "fsx_stream_wait_batches": (C.c_int, [vp, vp, C.c_int]),
        "fsx_verdict_batch": (C.c_int, [vp, u8p, u8p, u8p, sz, u8p]),
        "fsx_verdict_batch_device": (C.c_int, [vp, vp, vp, vp, sz, vp]),
        "fsx_process_batch_device": (C.c_int, [vp, vp, vp, vp, sz, vp, vp, vp, vp, vp, vp, sz]),
        "fsx_verdict_records_device": (C.c_int, [vp, vp, sz, C.c_uint32, vp]),
        "fsx_map_update_batch": (C.c_int, [vp, C.c_int, vp, vp, sz, C.c_uint64]),
        "fsx_process_records_device": (C.c_int, [vp, vp, sz, C.c_uint32, vp, vp, vp, vp, vp, vp, sz]),
        "fsx_map_lookup": (C.c_int, [vp, C.c_int, vp, vp]),
        "fsx_map_update": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint64]),
        "fsx_map_delete": (C.c_int, [vp, C.c_int, vp]),
        "fsx_map_dump": (C.c_int, [vp, C.c_int, vp, vp, sz, C.POINTER(sz)]),
        "fsx_get_stats": (C.c_int, [vp, C.POINTER(FsxStats)]),
        "fsx_reset": (C.c_int, [vp]),
        "fsx_load_q8_model": (C.c_int, [vp, C.POINTER(FsxQ8Model)]),
        "fsx_score": (C.c_int, [vp, vp, sz, vp, vp]),
        "fsx_score_device": (C.c_int, [vp, vp, sz, vp, vp]),
        "fsx_flow_features": (C.c_int, [vp, vp, vp, vp, sz, sz, vp, vp, vp, C.POINTER(sz)]),
        "fsx_flows_begin": (C.c_int, [vp]),
        "fsx_flows_end": (C.c_int, [vp, vp, vp, vp, vp, vp, sz, vp]),
        "fsx_flow_partials_records_device": (C.c_int, [vp, vp, sz, C.c_uint32, C.c_uint32, vp, sz, vp]),
        "fsx_flows_merge_device": (C.c_int, [vp, vp, sz]),
        "fsx_flows_merge_counted_device": (C.c_int, [vp, vp, sz, vp]),
        "fsx_shard_pack_filtered_device": (C.c_int, [vp, vp, vp, vp, sz, C.c_uint32, C.c_uint32, vp, vp, vp,
                                                     vp, vp]),
        "fsx_shard_filter_plan_device": (C.c_int, [vp, vp, C.c_uint32, C.c_uint32, vp]),
        "fsx_blocklist_replica_blocks_device": (C.c_int, [vp, vp, C.c_uint32, sz]),
        "fsx_last_timings": (C.c_int, [vp, vp, vp, vp, C.c_int, C.c_int, C.POINTER(C.c_int)]),
        "fsx_enable_timing": (C.c_int, [vp, C.c_int]),
        "fsx_last_batch_info": (C.c_int, [vp, vp, C.c_int]),
        "fsx_shard_owner": (C.c_uint32, [vp, C.c_int, C.c_uint32]),
        "fsx_shard_pack_device": (C.c_int, [vp, vp, vp, vp, sz, C.c_uint32, C.c_uint32, vp, vp,
                                            vp, vp]),
        "fsx_shard_clock_device": (C.c_int, [vp, vp, sz, vp]),
        "fsx_blocklist_export_device": (C.c_int, [vp, vp, sz, vp]),
        "fsx_blocklist_replica_device": (C.c_int, [vp, vp, sz]),
        "fsx_shard_unpack_device": (C.c_int, [vp, vp, sz, vp, vp, vp]),
        "fsx_shard_unpack16_device": (C.c_int, [vp, vp, sz, vp, vp, vp]),
        "fsx_shard_scatter_device": (C.c_int, [vp, vp, vp, sz, vp]),
        "fsx_shard_scatter_regions_device": (C.c_int, [vp, vp, vp, sz, sz, vp, C.c_uint32, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


# Every symbol include/fsx_hip.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = [
    "fsx_abi_version", "fsx_config_default", "fsx_open", "fsx_close", "fsx_last_error",
    "fsx_set_stream", "fsx_sync", "fsx_set_pipeline", "fsx_stream_wait_batches", "fsx_verdict_batch", "fsx_verdict_batch_device",
    "fsx_process_batch_device", "fsx_verdict_records_device", "fsx_process_records_device",
    "fsx_map_lookup", "fsx_map_update", "fsx_map_update_batch", "fsx_map_delete", "fsx_map_dump",
    "fsx_get_stats",
    "fsx_reset", "fsx_load_q8_model", "fsx_score", "fsx_score_device", "fsx_flow_features",
    "fsx_flows_begin", "fsx_flows_end", "fsx_flow_partials_records_device", "fsx_flows_merge_device",
    "fsx_flows_merge_counted_device", "fsx_shard_pack_filtered_device", "fsx_shard_filter_plan_device",
    "fsx_blocklist_replica_blocks_device",
    "fsx_last_timings", "fsx_enable_timing", "fsx_last_batch_info",
    "fsx_shard_owner", "fsx_shard_pack_device", "fsx_shard_unpack_device", "fsx_shard_unpack16_device",
    "fsx_shard_scatter_device", "fsx_shard_scatter_regions_device", "fsx_shard_clock_device", "fsx_blocklist_export_device",
    "fsx_blocklist_replica_device", "fsx_pcap_index", "fsx_pcap_records_device",
]

SHARD_RECORD_BYTES = 32
SHARD_RECORD16_BYTES = 16
SHARD_PACK_ERR = 1   # counts[G + 1] of a pack whose device placement failed (FSX_SHARD_PACK_ERR)
SHARD_BLOCK_BYTES = 32
SHARD_FILTER_BLOCKLIST = 1
SHARD_COMPACT = 2
SHARD_DROP_RECORDS = 4
SHARD_REGIONS = 8
FLOW_PARTIAL_BYTES = 112
MAX_SHARDS = 64


def shard_owner(key16: bytes, family: int, n_shards: int) -> int:
    """Owner rank of a source (include/fsx_hip.h fsx_shard_owner; host-only)."""
    k = bytes(key16).ljust(16, b"\0")
    return int(load_library().fsx_shard_owner(k, int(family), int(n_shards)))


def default_config(**overrides) -> FsxConfig:
    lib = load_library()
    cfg = FsxConfig()
    lib.fsx_config_default(C.byref(cfg))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown config field {k}")
        setattr(cfg, k, v)
    return cfg


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


_V6_MAPS = (MAP_IPV6_STATS, MAP_IPV6_BLACKLIST, MAP_IPV6_TOKENS)


def _key_len(map_id: int) -> int:
    if map_id == MAP_IPV4_PREFIX:
        return 8
    if map_id == MAP_IPV6_PREFIX:
        return 20
    return 16 if map_id in _V6_MAPS else 4


def prefix_key(addr: bytes, prefixlen: int) -> bytes:
    """struct bpf_lpm_trie_key {u32 prefixlen; u8 addr[4 | 16]} of a prefix-map key."""
    addr = bytes(addr)
    if len(addr) not in (4, 16):
        raise ValueError("prefix addresses are 4 or 16 bytes")
    return int(prefixlen).to_bytes(4, "little") + addr


def _value_words(map_id: int) -> int:
    """u64 words of a per-IP map value: ip_stats 3, token-bucket state 2, blacklist 1."""
    if map_id in (MAP_IPV4_STATS, MAP_IPV6_STATS):
        return 3
    if map_id in (MAP_IPV4_TOKENS, MAP_IPV6_TOKENS):
        return 2
    return 1


def _key_bytes(map_id: int, key) -> bytes:
    if isinstance(key, int):
        key = key.to_bytes(4, "little")
    key = bytes(key)
    want = _key_len(map_id)
    if len(key) != want:
        raise ValueError(f"{MAP_NAMES[map_id]} keys are {want} bytes")
    return key


class FsxContext:
    """One data-plane instance (the XDP program + its five maps) on one GPU."""

    def __init__(self, config: FsxConfig | None = None, **overrides):
        self._lib = load_library()
        self.config = config if config is not None else default_config(**overrides)
        h = C.c_void_p()
        rc = self._lib.fsx_open(C.byref(h), C.byref(self.config))
        if rc != 0:
            raise FsxError(rc, "fsx_open failed (no GPU or bad config)")
        self._h = h

    # -- plumbing
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self._lib.fsx_last_error(self._h)
            raise FsxError(rc, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fsx_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self._check(self._lib.fsx_sync(self._h), "fsx_sync")

    def set_pipeline(self, on: bool | int = True):
        """Batch pipelining (include/fsx_hip.h fsx_set_pipeline): the next batch's parse and
        sort overlap this batch's walkers and verdicts; read outputs after sync(). on = 2:
        batches whole on the context stream, only without a host synchronization per call."""
        self._check(self._lib.fsx_set_pipeline(self._h, int(on)), "fsx_set_pipeline")

    def stream_wait_batches(self, stream_handle: int, all_batches: bool = True):
        """hip_stream waits for the batches enqueued so far (include/fsx_hip.h
        fsx_stream_wait_batches): all_batches=False leaves out the last split batch, whose
        tail the next batch call enqueues."""
        self._check(self._lib.fsx_stream_wait_batches(self._h, stream_handle, int(bool(all_batches))),
                    "fsx_stream_wait_batches")

    def set_stream(self, stream_handle: int | None):
        self._check(self._lib.fsx_set_stream(self._h, stream_handle or None), "fsx_set_stream")

    # -- verdict path
    def verdict_batch(self, hdr: np.ndarray, length: np.ndarray, ts: np.ndarray) -> np.ndarray:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, HDR_BYTES)
        n = hdr.shape[0]
        length = np.ascontiguousarray(length, dtype=np.uint32)
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        if length.shape != (n,) or ts.shape != (n,):
            raise ValueError("hdr, len and ts must describe the same packets")
        out = np.empty(n, dtype=np.uint8)
        if n:
            self._check(self._lib.fsx_verdict_batch(self._h, _ptr(hdr), _ptr(length), _ptr(ts),
                                                    n, _ptr(out)), "fsx_verdict_batch")
        return out

    def verdict_batch_device(self, d_hdr: int, d_len: int, d_ts: int, n: int, d_verdict: int):
        self._check(self._lib.fsx_verdict_batch_device(self._h, d_hdr, d_len, d_ts, n, d_verdict),
                    "fsx_verdict_batch_device")

    def process_batch_device(self, d_hdr: int, d_len: int, d_ts: int, n: int, d_verdict: int,
                             d_keys16: int, d_family: int, d_features: int | None, d_prob: int | None,
                             d_malicious: int | None, flow_cap: int):
        """Verdicts + per-source features + q8 scores (device pointers, asynchronous)."""
        self._check(self._lib.fsx_process_batch_device(self._h, d_hdr, d_len, d_ts, n, d_verdict,
                                                       d_keys16, d_family, d_features, d_prob,
                                                       d_malicious, flow_cap),
                    "fsx_process_batch_device")

    def verdict_records_device(self, d_records: int, n: int, rec_bytes: int, d_verdict: int):
        """Owner side of the sharded path: the pipeline on n exchange records (asynchronous)."""
        self._check(self._lib.fsx_verdict_records_device(self._h, d_records, n, rec_bytes, d_verdict),
                    "fsx_verdict_records_device")

    def process_records_device(self, d_records: int, n: int, rec_bytes: int, d_verdict: int,
                               d_keys16: int, d_family: int, d_features: int | None,
                               d_prob: int | None, d_malicious: int | None, flow_cap: int):
        self._check(self._lib.fsx_process_records_device(self._h, d_records, n, rec_bytes, d_verdict,
                                                         d_keys16, d_family, d_features, d_prob,
                                                         d_malicious, flow_cap),
                    "fsx_process_records_device")

    # -- maps (bpf_map_*_elem)
    def map_lookup(self, map_id: int, key):
        if map_id == MAP_STATS:
            v = (C.c_uint64 * 2)()
            self._check(self._lib.fsx_map_lookup(self._h, map_id, C.byref(C.c_uint32(0)), v),
                        "map_lookup")
            return tuple(v)
        k = _key_bytes(map_id, key)
        v = (C.c_uint64 * 3)()
        rc = self._lib.fsx_map_lookup(self._h, map_id, k, v)
        if rc == -errno.ENOENT:
            return None
        self._check(rc, "map_lookup")
        vw = _value_words(map_id)
        return tuple(v[:vw]) if vw > 1 else int(v[0])

    def map_update(self, map_id: int, key, value, flags: int = BPF_ANY):
        if map_id == MAP_STATS:
            v = (C.c_uint64 * 2)(*value)
            self._check(self._lib.fsx_map_update(self._h, map_id, C.byref(C.c_uint32(int(key))), v,
                                                 flags), "map_update")
            return
        k = _key_bytes(map_id, key)
        vw = _value_words(map_id)
        if vw > 1:
            v = (C.c_uint64 * vw)(*value)
        else:
            v = (C.c_uint64 * 1)(int(value))
        self._check(self._lib.fsx_map_update(self._h, map_id, k, v, flags), "map_update")

    def map_update_batch(self, map_id: int, entries: dict):
        """BPF_MAP_UPDATE_BATCH (BPF_ANY) of {key: value} in the map's layouts (the dict
        map_dump returns): one device pass; all or nothing (-ENOSPC when full)."""
        if map_id == MAP_STATS:
            raise ValueError("stats_map has no batched update")
        klen = _key_len(map_id)
        vw = _value_words(map_id)
        n = len(entries)
        keys = np.zeros((max(n, 1), klen), dtype=np.uint8)
        vals = np.zeros((max(n, 1), vw), dtype=np.uint64)
        for i, (k, v) in enumerate(entries.items()):
            keys[i] = np.frombuffer(_key_bytes(map_id, k), dtype=np.uint8)
            vals[i] = v if vw > 1 else [int(v)]
        self._check(self._lib.fsx_map_update_batch(self._h, map_id, _ptr(keys), _ptr(vals), n, BPF_ANY),
                    "map_update_batch")

    def map_update_arrays(self, map_id: int, keys: np.ndarray, values: np.ndarray):
        """map_update_batch from arrays: keys [n, klen] u8, values [n] or [n, words] u64."""
        klen, vw = _key_len(map_id), _value_words(map_id)
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, klen)
        v = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, vw)
        if k.shape[0] != v.shape[0]:
            raise ValueError("keys and values differ in length")
        self._check(self._lib.fsx_map_update_batch(self._h, map_id, _ptr(k), _ptr(v), k.shape[0], BPF_ANY),
                    "map_update_batch")

    def map_count(self, map_id: int) -> int:
        """Entries of one map (fsx_map_dump with no buffers)."""
        n = C.c_size_t()
        self._check(self._lib.fsx_map_dump(self._h, map_id, None, None, 0, C.byref(n)), "map_dump")
        return int(n.value)

    def map_delete(self, map_id: int, key) -> bool:
        rc = self._lib.fsx_map_delete(self._h, map_id, _key_bytes(map_id, key))
        if rc == -errno.ENOENT:
            return False
        self._check(rc, "map_delete")
        return True

    def map_dump(self, map_id: int) -> dict:
        n = C.c_size_t()
        self._check(self._lib.fsx_map_dump(self._h, map_id, None, None, 0, C.byref(n)), "map_dump")
        cap = n.value
        if map_id == MAP_STATS:
            return {0: self.map_lookup(MAP_STATS, 0)}
        klen = _key_len(map_id)
        vw = _value_words(map_id)
        keys = np.zeros((max(cap, 1), klen), dtype=np.uint8)
        vals = np.zeros((max(cap, 1), vw), dtype=np.uint64)
        self._check(self._lib.fsx_map_dump(self._h, map_id, _ptr(keys), _ptr(vals), cap, C.byref(n)),
                    "map_dump")
        m = min(cap, n.value)
        out = {}
        for i in range(m):
            out[keys[i].tobytes()] = tuple(int(x) for x in vals[i]) if vw > 1 else int(vals[i, 0])
        return out

    def map_arrays(self, map_id: int):
        """(keys [n, klen] u8, values [n, words] u64) of one per-IP map, unordered: the
        array form of map_dump for maps of millions of entries."""
        n = C.c_size_t()
        self._check(self._lib.fsx_map_dump(self._h, map_id, None, None, 0, C.byref(n)), "map_dump")
        cap = n.value
        keys = np.zeros((max(cap, 1), _key_len(map_id)), dtype=np.uint8)
        vals = np.zeros((max(cap, 1), _value_words(map_id)), dtype=np.uint64)
        self._check(self._lib.fsx_map_dump(self._h, map_id, _ptr(keys), _ptr(vals), cap, C.byref(n)),
                    "map_dump")
        m = min(cap, n.value)
        return keys[:m], vals[:m]

    def stats(self) -> tuple[int, int]:
        s = FsxStats()
        self._check(self._lib.fsx_get_stats(self._h, C.byref(s)), "fsx_get_stats")
        return int(s.allowed), int(s.dropped)

    def reset(self):
        self._check(self._lib.fsx_reset(self._h), "fsx_reset")

    # -- scoring
    def load_q8_model(self, model: FsxQ8Model):
        self._check(self._lib.fsx_load_q8_model(self._h, C.byref(model)), "fsx_load_q8_model")

    def score(self, features: np.ndarray):
        f = np.ascontiguousarray(features, dtype=np.float32).reshape(-1, 8)
        n = f.shape[0]
        p = np.empty(n, dtype=np.float32)
        d = np.empty(n, dtype=np.uint8)
        if n:
            self._check(self._lib.fsx_score(self._h, _ptr(f), n, _ptr(p), _ptr(d)), "fsx_score")
        return p, d

    def score_device(self, d_feat: int, n: int, d_prob: int, d_dec: int):
        self._check(self._lib.fsx_score_device(self._h, d_feat, n, d_prob, d_dec), "fsx_score_device")

    def flow_features(self, hdr: np.ndarray, length: np.ndarray, ts: np.ndarray):
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8).reshape(-1, HDR_BYTES)
        n = hdr.shape[0]
        length = np.ascontiguousarray(length, dtype=np.uint32)
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        keys = np.zeros((max(n, 1), 16), dtype=np.uint8)
        fam = np.zeros(max(n, 1), dtype=np.uint8)
        feat = np.zeros((max(n, 1), 8), dtype=np.float32)
        nf = C.c_size_t()
        self._check(self._lib.fsx_flow_features(self._h, _ptr(hdr), _ptr(length), _ptr(ts), n,
                                                max(n, 1), _ptr(keys), _ptr(fam), _ptr(feat),
                                                C.byref(nf)), "fsx_flow_features")
        m = nf.value
        return keys[:m], fam[:m], feat[:m]

    def flows_begin(self):
        """Start accumulating one global batch's per-source sums over several calls."""
        self._check(self._lib.fsx_flows_begin(self._h), "fsx_flows_begin")

    def flows_end(self, d_keys16: int, d_family: int, d_features: int | None, d_prob: int | None,
                  d_malicious: int | None, cap: int, d_rows: int | None):
        """Rows of every source accumulated since flows_begin (device pointers, async)."""
        self._check(self._lib.fsx_flows_end(self._h, d_keys16, d_family, d_features, d_prob,
                                            d_malicious, cap, d_rows), "fsx_flows_end")

    def flow_partials_records_device(self, d_records: int, n: int, rec_bytes: int, n_shards: int,
                                     d_partials: int, cap_per_shard: int, d_counts: int):
        """Flow partial (raw sums, first / last ts) of every source of n records, into the run
        of its owner (n_shards runs of cap_per_shard; d_counts[o] per run). No map state."""
        self._check(self._lib.fsx_flow_partials_records_device(self._h, d_records, n, rec_bytes, n_shards,
                                                               d_partials, cap_per_shard, d_counts),
                    "fsx_flow_partials_records_device")

    def flows_merge_device(self, d_partials: int, m: int):
        """Between flows_begin and flows_end: merge m partials (distinct sources) in order."""
        self._check(self._lib.fsx_flows_merge_device(self._h, d_partials, m), "fsx_flows_merge_device")

    BATCH_INFO = ("ip_packets", "sources", "new_sources", "any_ipv6", "non_monotone",
                  "max_len", "max_ts", "allowed", "dropped", "prefix_rule_drops", "sorted_payload",
                  "light_packets", "evicted", "heavy_unsorted", "admitted", "transient",
                  "hfast_batches", "hrun_batches", "ordered_inserts")

    def last_batch_info(self) -> dict:
        buf = (C.c_uint64 * len(self.BATCH_INFO))()
        rc = self._lib.fsx_last_batch_info(self._h, buf, len(self.BATCH_INFO))
        if rc < 0:
            self._check(rc, "fsx_last_batch_info")
        return {k: int(buf[i]) for i, k in enumerate(self.BATCH_INFO[:rc])}

    # -- sharding (SURVEY.md §8 e; protocol in flowsentryx_amd/shard.py)
    def shard_pack_device(self, d_hdr: int, d_len: int, d_ts: int, n: int, n_shards: int,
                          d_verdict: int, d_records: int, d_send_idx: int, d_counts: int,
                          flags: int = 0):
        self._check(self._lib.fsx_shard_pack_device(self._h, d_hdr, d_len, d_ts, n, n_shards,
                                                    flags, d_verdict, d_records, d_send_idx,
                                                    d_counts), "fsx_shard_pack_device")

    def shard_pack_filtered_device(self, d_hdr: int, d_len: int, d_ts: int, n: int, n_shards: int,
                                   d_filter: int, d_verdict: int, d_records: int, d_send_idx: int,
                                   d_counts: int, flags: int = 0):
        """shard_pack_device with the replica filter iff the device word *d_filter != 0."""
        self._check(self._lib.fsx_shard_pack_filtered_device(self._h, d_hdr, d_len, d_ts, n, n_shards, flags,
                                                             d_filter, d_verdict, d_records, d_send_idx,
                                                             d_counts), "fsx_shard_pack_filtered_device")

    def shard_filter_plan_device(self, d_clocks: int, n_shards: int, k: int, d_filter: int):
        self._check(self._lib.fsx_shard_filter_plan_device(self._h, d_clocks, n_shards, k, d_filter),
                    "fsx_shard_filter_plan_device")

    def blocklist_replica_blocks_device(self, d_blocks: int, n_blocks: int, cap: int):
        self._check(self._lib.fsx_blocklist_replica_blocks_device(self._h, d_blocks, n_blocks, cap),
                    "fsx_blocklist_replica_blocks_device")

    def flows_merge_counted_device(self, d_partials: int, cap: int, d_count: int):
        """Between flows_begin and flows_end: merge min(*d_count, cap) partials (device count)."""
        self._check(self._lib.fsx_flows_merge_counted_device(self._h, d_partials, cap, d_count),
                    "fsx_flows_merge_counted_device")

    def shard_clock_device(self, d_ts: int, n: int, d_out3: int):
        self._check(self._lib.fsx_shard_clock_device(self._h, d_ts, n, d_out3),
                    "fsx_shard_clock_device")

    def blocklist_export_device(self, d_entries: int, cap: int, d_count: int):
        self._check(self._lib.fsx_blocklist_export_device(self._h, d_entries, cap, d_count),
                    "fsx_blocklist_export_device")

    def blocklist_replica_device(self, d_entries: int, m: int):
        self._check(self._lib.fsx_blocklist_replica_device(self._h, d_entries, m),
                    "fsx_blocklist_replica_device")

    def shard_unpack_device(self, d_records: int, m: int, d_hdr: int, d_len: int, d_ts: int,
                            rec_bytes: int = SHARD_RECORD_BYTES):
        fn = "fsx_shard_unpack16_device" if rec_bytes == SHARD_RECORD16_BYTES else "fsx_shard_unpack_device"
        self._check(getattr(self._lib, fn)(self._h, d_records, m, d_hdr, d_len, d_ts), fn)

    def shard_scatter_device(self, d_ret: int, d_send_idx: int, m: int, d_verdict: int):
        self._check(self._lib.fsx_shard_scatter_device(self._h, d_ret, d_send_idx, m, d_verdict),
                    "fsx_shard_scatter_device")

    def shard_scatter_regions_device(self, d_ret: int, d_send_idx: int, m: int, region: int, d_counts: int,
                                     n_shards: int, d_verdict: int):
        """fsx_shard_scatter_regions_device: m verdicts owner by owner back through a
        FSX_SHARD_REGIONS pack's send indices (regions of `region` entries, its counts)."""
        self._check(self._lib.fsx_shard_scatter_regions_device(self._h, d_ret, d_send_idx, m, region, d_counts,
                                                               n_shards, d_verdict),
                    "fsx_shard_scatter_regions_device")

    # -- timing
    def enable_timing(self, on: bool = True):
        self._check(self._lib.fsx_enable_timing(self._h, int(on)), "fsx_enable_timing")

    def last_timings(self) -> list[tuple[str, float, float]]:
        """[(kernel, ms per batch, launches per batch)] since the previous call."""
        cap, nl = 48, 32
        ms = (C.c_float * cap)()
        nlaunch = (C.c_float * cap)()
        names = C.create_string_buffer(cap * nl)
        cnt = C.c_int()
        self._check(self._lib.fsx_last_timings(self._h, ms, nlaunch, names, cap, nl, C.byref(cnt)),
                    "fsx_last_timings")
        raw = names.raw
        return [(raw[i * nl:(i + 1) * nl].split(b"\0")[0].decode(), float(ms[i]), float(nlaunch[i]))
                for i in range(cnt.value)]


def ipv4_key(addr: str) -> bytes:
    """Map key of an IPv4 source: the raw saddr bytes (network order)."""
    return bytes(int(x) for x in addr.split("."))
