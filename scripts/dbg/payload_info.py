"""Debug: last_batch_info of test_sorted_payload_and_gather_paths' input (dt = 1)."""
import sys
sys.path[:0] = [".", "tests"]
import numpy as np
from test_gpu_parity import rand_stream, _with_far_nonip, CFGS
from flowsentryx_amd import lib
rng = np.random.default_rng(77)
hdr, ln, ts = rand_stream(rng, 40000, 400, dt_max=400, v6_frac=0.25, t0=10**12)
hdr, ln, ts = _with_far_nonip(hdr, ln, ts, 1)
print("host: min", int(ts.min()), "ts0", int(ts[0]), "max", int(ts.max()), "mono", bool((np.diff(ts.astype(np.int64)) >= 0).all()))
for name in ("tight",):
    with lib.FsxContext(max_batch=len(ln), max_entries=1 << 18, **CFGS[name]) as c:
        c.verdict_batch(hdr, ln, ts)
        print(name, c.last_batch_info())
