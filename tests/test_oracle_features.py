"""CPU: the build-defined flow features of the oracle on hand-computed
cases (parity unpinned: the reference has no feature code, src/fsx_kern_ml.c)."""
import math

import numpy as np

from flowsentryx_amd import synth


def test_three_packet_flow(oracle):
    src = bytes([192, 0, 2, 9])
    frames = [synth.frame_ipv4_udp(src, L, dport=443) for L in (100, 200, 600)]
    hdr = synth.records(frames)
    ln = np.array([100, 200, 600], np.uint32)
    ts = np.array([1_000_000, 3_000_000, 7_000_000], np.uint64)  # IATs 2 ms, 4 ms
    keys, fam, feat = oracle.flow_features(hdr, ln, ts)
    assert list(fam) == [4] and keys[0, :4].tobytes() == src
    mean = 300.0
    var = ((100 - mean) ** 2 + (200 - mean) ** 2 + (600 - mean) ** 2) / 2
    iat = [2000.0, 4000.0]  # microseconds
    iat_std = math.sqrt(((2000 - 3000) ** 2 + (4000 - 3000) ** 2) / 1)
    want = np.array([443, mean, math.sqrt(var), var, mean, 3000.0, iat_std, 4000.0], np.float32)
    assert np.array_equal(feat[0], want)


def test_single_packet_and_non_ip(oracle):
    hdr = synth.records([synth.frame_raw(0x0806, bytes(40), 60),
                         synth.frame_ipv6_udp(bytes(range(16)), 80, dport=53)])
    keys, fam, feat = oracle.flow_features(hdr, np.array([60, 80], np.uint32),
                                           np.array([5, 9], np.uint64))
    assert list(fam) == [6]
    assert np.array_equal(feat[0], np.array([53, 80, 0, 0, 80, 0, 0, 0], np.float32))
