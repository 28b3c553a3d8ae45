"""Debug: GPU vs oracle flow rows of test_flow_features_random's stream, field by field."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
torch.cuda.init()
from test_gpu_parity import rand_stream, _sorted_flows
from flowsentryx_amd import lib
from oracle import pyoracle as oracle
rng = np.random.default_rng(31)
hdr, ln, ts = rand_stream(rng, 60000, 700, dt_max=5000, v6_frac=0.3, nonip_frac=0.02, short_frac=0.01)
ko, fo, xo = oracle.flow_features(hdr, ln, ts)
with lib.FsxContext() as c:
    kg, fg, xg = c.flow_features(hdr, ln, ts)
ko, fo, xo = _sorted_flows(ko, fo, xo)
kg, fg, xg = _sorted_flows(kg, fg, xg)
bad = np.nonzero((xg.view(np.uint32) != xo.view(np.uint32)).any(axis=1))[0]
print("rows", len(fo), "bad", bad.size)
fields = (xg.view(np.uint32) != xo.view(np.uint32)).sum(axis=0)
print("bad per field", fields)
for i in bad[:6]:
    print(i, fo[i], "gpu", xg[i], "\n   ora", xo[i])
