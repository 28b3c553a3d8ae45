"""Per-kernel split of warm owner record batches (debug for scripts/shard_kernels.py)."""
import json
import sys
import time

import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from flowsentryx_amd import lib, synth  # noqa: E402
from flowsentryx_amd.shard import HipShardEngine  # noqa: E402

p, s = synth.config_params(2)
n = int(p.n)
dev = torch.device("cuda", 0)
hdr = torch.empty(n * 64, dtype=torch.uint8, device=dev)
ln = torch.empty(n, dtype=torch.int32, device=dev)
ts = torch.empty(n, dtype=torch.int64, device=dev)
v = torch.empty(n, dtype=torch.uint8, device=dev)
synth.generate_device(p, s, 0, n, hdr.data_ptr(), ln.data_ptr(), ts.data_ptr())
torch.cuda.synchronize()
with lib.FsxContext(max_batch=n, max_entries=int(p.n_ips), device=0) as c0:
    e = HipShardEngine(c0, n, dev)
    with e.stream_ctx():
        rec, counts = e.pack(hdr, ln, ts, n, 1, v)
    c0.sync()
    m, rb = int(counts[0].item()), int(counts[2].item())
    rec = rec.clone()
tsw = rec[:m * rb].view(torch.int64)[1::2]
dur = int(p.duration_ns)
ov = torch.empty(m, dtype=torch.uint8, device=dev)
with lib.FsxContext(max_batch=n, max_entries=int(p.n_ips), device=0) as ctx:
    if len(sys.argv) > 1:
        ctx.set_pipeline(int(sys.argv[1]))
    for it in range(4):
        tsw.add_(dur)
        torch.cuda.synchronize()
        if it == 3 and len(sys.argv) == 1:
            ctx.enable_timing(True)
        t0 = time.perf_counter()
        ctx.verdict_records_device(rec.data_ptr(), m, rb, ov.data_ptr())
        ctx.sync()
        print(it, "ms", (time.perf_counter() - t0) * 1e3, ctx.last_batch_info(), flush=True)
    if len(sys.argv) == 1:
        print(json.dumps([(a, round(b, 4)) for a, b, _ in ctx.last_timings()]))
