"""Write tests/golden/kat_fixed_window.json: known-answer tests of the REFERENCE program.

Each case is a packet sequence and the verdicts / map values the reference's own
src/fsx_kern.o produced for it under BPF_PROG_TEST_RUN with a deterministic clock,
as recorded by the survey (SURVEY.md §4 "Known-answer tests ... all observed",
and §8 a1/a3 derived facts). Expectations are transcribed from those observations,
NOT computed by this repo's oracle. Runs: {"src": ip, "family": 4|6, "len": L,
"count": k, "t0": ns, "dt": ns, "expect": [verdict per packet] or a single code}.
"""
import json
from pathlib import Path

DROP, PASS = 1, 2
T0 = 5_000_000_000
cases = []

# 1. a fresh IP passes packets 1..1000 of a window; the 1001st (within 1 s) drops and
#    blacklists until t + 10e9 (SURVEY.md §4 item 1, §8 a3 "derived facts").
cases.append({
    "name": "fresh_ip_1000_pass_then_drop",
    "runs": [{"src": "10.1.0.1", "family": 4, "len": 100, "count": 1001, "t0": T0, "dt": 1000,
              "expect": [PASS] * 1000 + [DROP]}],
    "maps": {"ipv4_blacklist_map": {"10.1.0.1": T0 + 1000 * 1000 + 10_000_000_000},
             "ipv4_stats_map": {"10.1.0.1": [1001, 100 * 1001, T0]}},
    "stats": [1000, 1],
})

# 2. blacklist expiry is inclusive: DROP at t == till, PASS at till + 1 (§4 item 2).
tk = T0 + 1000 * 1000
till = tk + 10_000_000_000
cases.append({
    "name": "blacklist_inclusive_expiry",
    "runs": [{"src": "10.1.0.2", "family": 4, "len": 100, "count": 1001, "t0": T0, "dt": 1000,
              "expect": [PASS] * 1000 + [DROP]},
             {"src": "10.1.0.2", "family": 4, "len": 100, "count": 1, "t0": till, "dt": 0,
              "expect": [DROP]},
             {"src": "10.1.0.2", "family": 4, "len": 100, "count": 1, "t0": till + 1, "dt": 0,
              "expect": [PASS]}],
    # the unblocked packet resets the window and is not counted (pps = 0)
    "maps": {"ipv4_stats_map": {"10.1.0.2": [0, 0, till + 1]}},
    "stats": [1001, 2],
})

# 3. window reset needs now - track_time > 1e9 strictly: a packet at exactly +1e9 is
#    counted (§4 item 3) — 999 packets near t0, then 2 at t0 + 1e9: the 1000th
#    (pps 1000) passes, the 1001st (pps 1001) drops.
cases.append({
    "name": "window_boundary_counted",
    "runs": [{"src": "10.1.0.3", "family": 4, "len": 100, "count": 999, "t0": T0, "dt": 1,
              "expect": PASS},
             {"src": "10.1.0.3", "family": 4, "len": 100, "count": 2, "t0": T0 + 1_000_000_000,
              "dt": 0, "expect": [PASS, DROP]}],
    "stats": [1000, 1],
})

# 4. ... and +1e9+1 resets: the reset packet passes with pps = 0, packets 2..1001 of
#    the new window pass, the next drops (§4 item 3, §8 a3).
cases.append({
    "name": "window_reset_strictly_greater",
    "runs": [{"src": "10.1.0.4", "family": 4, "len": 100, "count": 999, "t0": T0, "dt": 1,
              "expect": PASS},
             {"src": "10.1.0.4", "family": 4, "len": 100, "count": 1002,
              "t0": T0 + 1_000_000_001, "dt": 10, "expect": [PASS] * 1001 + [DROP]}],
    "stats": [2000, 1],
})

# 5. short / edge frames (§4 item 4; the 13-byte case is restatement-only because
#    BPF_PROG_TEST_RUN rejects frames < 14 B). Parse drops and non-IP passes are
#    never counted in stats_map.
cases.append({
    "name": "edge_frames",
    "frames": [
        {"kind": "ipv4", "src": "10.2.0.1", "len": 14, "expect": DROP},
        {"kind": "ipv4", "src": "10.2.0.1", "len": 33, "expect": DROP},
        {"kind": "ipv4", "src": "10.2.0.1", "len": 34, "expect": PASS},
        {"kind": "ipv6", "src": "2001:db8::77", "len": 53, "expect": DROP},
        {"kind": "raw", "proto": 0x0806, "len": 60, "expect": PASS},
        {"kind": "raw", "proto": 0x8100, "len": 60, "expect": PASS},
        {"kind": "ipv4_v6ihl15", "src": "10.2.0.2", "len": 60, "expect": PASS},
        {"kind": "ipv4", "src": "10.2.0.3", "len": 13, "expect": DROP, "restatement_only": True},
    ],
    "stats": [2, 0],
})

out = Path(__file__).with_name("kat_fixed_window.json")
out.write_text(json.dumps({"source": "SURVEY.md §4 / §8 a1,a3 (observed on src/fsx_kern.o)",
                           "XDP_DROP": DROP, "XDP_PASS": PASS, "cases": cases}, indent=1) + "\n")
print("wrote", out)
