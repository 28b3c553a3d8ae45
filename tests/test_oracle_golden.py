"""CPU: the oracle against every golden fixture the reference path has.

* parse  — tests/golden/parse_vectors.npz, produced by the reference's own
  src/parsing_helper.h (oracle/_ref), plus a live cross-check when oracle/_ref exists;
* fixed window — the survey's observed known-answer tests (kat_fixed_window.json);
* scoring — torch-produced vectors with the reference weights and random models.
"""
import json

import numpy as np
import pytest

from kat import GOLDEN, build_case, expected_maps, load_kats


def test_parse_matches_reference_parsers(oracle):
    g = np.load(GOLDEN / "parse_vectors.npz")
    cls, keys = oracle.parse(g["hdr"], g["len"])
    assert np.array_equal(cls, g["cls"])
    ip = g["cls"] >= 2
    assert np.array_equal(keys[ip], g["keys"][ip])


def test_parse_live_reference_random(oracle):
    if not oracle.REF_LIB.exists():
        pytest.skip("oracle/_ref not built (reference tree absent)")
    rng = np.random.default_rng(99)
    hdr = rng.integers(0, 256, (20000, 64), dtype=np.uint8)
    hdr[::3, 12:14] = (0x08, 0x00)
    hdr[1::3, 12:14] = (0x86, 0xDD)
    ln = rng.integers(0, 120, 20000).astype(np.uint32)
    a = oracle.parse(hdr, ln)
    b = oracle.ref_parse(hdr, ln)
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[1][a[0] >= 2], b[1][b[0] >= 2])


@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_oracle_known_answers(oracle, case):
    hdr, ln, ts, exp = build_case(case)
    o = oracle.Oracle(max_entries=1000)
    v = o.batch(hdr, ln, ts)
    assert np.array_equal(v, exp), np.nonzero(v != exp)[0][:10]
    assert list(o.stats()) == case["stats"]
    for mid, entries in expected_maps(case).items():
        dump = o.map_dump(mid)
        for k, val in entries.items():
            assert dump.get(k) == val, (mid, k, dump.get(k), val)


def test_score_reference_model(oracle):
    g = np.load(GOLDEN / "score_vectors.npz")
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    p, d, lq = oracle.score(ref, g["x_ref"])
    assert np.array_equal(lq, g["lq_ref"])
    assert np.array_equal(p.view(np.uint32), g["p_ref"].view(np.uint32))
    assert np.array_equal(d, (g["p_ref"] > 0.5).astype(np.uint8))


def test_score_closed_form_reference_weights(oracle):
    """for the shipped weights, malicious <=> acc >= 80, p in {0, .5, 255/256}."""
    g = np.load(GOLDEN / "score_vectors.npz")
    ref = json.loads((GOLDEN / "model_weights.json").read_text())
    p, d, lq = oracle.score(ref, g["x_ref"])
    assert set(np.unique(p).tolist()) <= {0.0, 0.5, 255 / 256}
    assert np.array_equal(d == 1, lq > 84)


def test_score_random_models(oracle):
    g = np.load(GOLDEN / "score_vectors.npz")
    models = json.loads((GOLDEN / "score_random_models.json").read_text())
    for i, m in enumerate(models):
        p, d, lq = oracle.score(m, g["rand_x"][i])
        assert np.array_equal(lq, g["rand_lq"][i]), i
        assert np.array_equal(p.view(np.uint32), g["rand_p"][i].view(np.uint32)), i


def test_sigmoid_lut(oracle):
    g = np.load(GOLDEN / "sigmoid_luts.npz")
    for s, z, lut in zip(g["scale"], g["zp"], g["lut"]):
        assert np.array_equal(oracle.sigmoid_lut(float(s), int(z)), lut), (s, z)
