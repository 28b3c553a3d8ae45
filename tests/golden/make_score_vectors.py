"""Generate the scoring golden fixtures with torch (build container only).

* model_weights.json  — the reference's src/model_weights.pth, loaded with
  torch.load(weights_only=True) (nothing executed from the file), flattened to the
  fsx_q8_model fields (include/fsx_hip.h).
* score_vectors.npz   — features and torch's outputs for the reference model
  (model/model.py:124-137 restated: QuantStub -> Linear(8,1) -> sigmoid ->
  DeQuantStub, default_qconfig, prepare_qat -> convert -> load_state_dict) plus
  random quantized models, engine x86 (torch 2.10 default).
* sigmoid_luts.npz    — torch's quantized sigmoid on all 256 inputs for random
  output qparams.
The restated module is 6 lines of torch; model/model.py itself is a training script
(it reads absent CSVs at import) and is not importable.
"""
import json
import sys
import warnings
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn
from torch.ao.quantization import DeQuantStub, QuantStub

warnings.filterwarnings("ignore")
HERE = Path(__file__).resolve().parent
REF_PTH = Path("/root/reference/src/model_weights.pth")
assert torch.backends.quantized.engine == "x86", torch.backends.quantized.engine


class LogisticRegression(nn.Module):  # model/model.py:124-137
    def __init__(self):
        super().__init__()
        self.quant = QuantStub()
        self.linear = nn.Linear(8, 1)
        self.dequant = DeQuantStub()

    def forward(self, x):
        return self.dequant(torch.sigmoid(self.linear(self.quant(x))))


def converted(state_dict):
    m = LogisticRegression()
    m.qconfig = torch.ao.quantization.default_qconfig
    m.train()
    mq = torch.ao.quantization.prepare_qat(m)
    mq.eval()
    mq = torch.ao.quantization.convert(mq)
    mq.load_state_dict(state_dict)
    return mq


def fields(mq):
    w = mq.linear.weight()
    return {
        "weight": [int(x) for x in w.int_repr().flatten().tolist()],
        "weight_scale": float(w.q_scale()),
        "bias": float(mq.linear.bias().detach().float()[0]),
        "in_scale": float(mq.quant.scale.item()),
        "in_zero_point": int(mq.quant.zero_point.item()),
        "out_scale": float(mq.linear.scale),
        "out_zero_point": int(mq.linear.zero_point),
    }


def run(mq, x):
    with torch.no_grad():
        p = mq(torch.from_numpy(x)).numpy().reshape(-1).astype(np.float32)
        lq = mq.linear(mq.quant(torch.from_numpy(x))).int_repr().numpy().reshape(-1).astype(np.uint8)
    return p, lq


def features(rng, n, ref):
    """Uniform over the CICIDS input ranges + boundary-biased + special values."""
    x = np.empty((n, 8), dtype=np.float32)
    x[:, 0] = rng.integers(0, 65536, n)
    x[:, 1:5] = rng.uniform(0, 1500, (n, 4))
    x[:, 5:8] = rng.uniform(0, 1.2e8, (n, 3))
    x[:, 3] = x[:, 2] ** 2
    m = n // 4  # boundary: near quantization half-steps of the input scale
    s = ref["in_scale"]
    k = rng.integers(0, 256, (m, 8))
    x[:m] = ((k + rng.choice([0.5, 0.49999, 0.50001, 0.0], (m, 8))) * s).astype(np.float32)
    sp = np.array([np.nan, np.inf, -np.inf, -1.0, 0.0, 1e30, -1e30, 3.0e8], dtype=np.float32)
    x[m:m + 64] = rng.choice(sp, (64, 8))
    return x


sd = torch.load(REF_PTH, weights_only=True)
ref_model = converted(sd)
ref = fields(ref_model)
(HERE / "model_weights.json").write_text(json.dumps(ref, indent=1) + "\n")

rng = np.random.default_rng(7)
x_ref = features(rng, 50000, ref)
p_ref, lq_ref = run(ref_model, x_ref)

rand_models, rand_x, rand_p, rand_lq = [], [], [], []
for t in range(12):
    f = {
        "weight": rng.integers(-128, 128, 8).tolist(),
        "weight_scale": float(np.float32(10 ** rng.uniform(-4, -1))),
        "bias": float(np.float32(rng.normal() * 10 ** rng.uniform(-2, 3))),
        "in_scale": float(np.float32(10 ** rng.uniform(-2, 6))),
        "in_zero_point": int(rng.integers(0, 256)),
        "out_scale": float(np.float32(10 ** rng.uniform(-3, 3))),
        "out_zero_point": int(rng.integers(0, 256)),
    }
    mq = converted(sd)
    wq = torch.quantize_per_tensor(torch.tensor(f["weight"], dtype=torch.float32).reshape(1, 8)
                                   * f["weight_scale"], f["weight_scale"], 0, torch.qint8)
    mq.linear.set_weight_bias(wq, torch.tensor([f["bias"]], dtype=torch.float32))
    mq.linear.scale = f["out_scale"]
    mq.linear.zero_point = f["out_zero_point"]
    mq.quant.scale = torch.tensor([f["in_scale"]])
    mq.quant.zero_point = torch.tensor([f["in_zero_point"]])
    f = fields(mq)
    x = features(rng, 4000, f)
    x[:, 1:] = rng.uniform(-3, 300, (4000, 7)).astype(np.float32) * f["in_scale"]
    p, lq = run(mq, x)
    rand_models.append(f); rand_x.append(x); rand_p.append(p); rand_lq.append(lq)

np.savez_compressed(HERE / "score_vectors.npz", x_ref=x_ref, p_ref=p_ref, lq_ref=lq_ref,
                    rand_x=np.stack(rand_x), rand_p=np.stack(rand_p), rand_lq=np.stack(rand_lq))
(HERE / "score_random_models.json").write_text(json.dumps(rand_models, indent=1) + "\n")

# quantized sigmoid tables
scales, zps, luts = [], [], []
lq = torch.arange(256, dtype=torch.uint8)
for t in range(400):
    so = float(np.float32(10 ** rng.uniform(-4, 6)))
    zp = int(rng.integers(0, 256))
    y = torch.sigmoid(torch._make_per_tensor_quantized_tensor(lq, so, zp))
    assert abs(y.q_scale() - 1 / 256) < 1e-12 and y.q_zero_point() == 0
    scales.append(so); zps.append(zp); luts.append(y.int_repr().numpy())
scales.append(ref["out_scale"]); zps.append(ref["out_zero_point"])
luts.append(torch.sigmoid(torch._make_per_tensor_quantized_tensor(lq, ref["out_scale"], ref["out_zero_point"])).int_repr().numpy())
np.savez_compressed(HERE / "sigmoid_luts.npz", scale=np.array(scales, dtype=np.float32),
                    zp=np.array(zps, dtype=np.int32), lut=np.stack(luts).astype(np.uint8))
dec = p_ref > 0.5
print(f"ref model {ref}\n{len(x_ref)} ref vectors, malicious {int(dec.sum())}, "
      f"p values {sorted(set(np.round(p_ref[~np.isnan(p_ref)], 6).tolist()))[:8]}")
