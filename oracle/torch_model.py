"""The reference model run by CPU PyTorch — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

model/model.py:124-137 restated (QuantStub -> Linear(8, 1) -> sigmoid -> DeQuantStub,
default_qconfig, prepare_qat -> convert), loaded with the fsx_q8_model fields of the
reference's src/model_weights.pth (tests/golden/model_weights.json, exported with
torch.load(weights_only=True) by tests/golden/make_score_vectors.py). This is the
"CPU PyTorch model.py" half of the reference CPU path that BASELINE.json's north_star
times beside the GPU (bench.py cpu_baseline.scoring) and the checker of the config-3
GPU scores. The product (flowsentryx_amd/) never imports it.
"""
from __future__ import annotations

import warnings

import numpy as np


def build(fields: dict):
    """The converted (int8) module with the given fsx_q8_model fields, engine x86."""
    import torch
    import torch.nn as nn
    from torch.ao.quantization import DeQuantStub, QuantStub

    warnings.filterwarnings("ignore")
    torch.backends.quantized.engine = "x86"

    class LogisticRegression(nn.Module):   # model/model.py:124-137
        def __init__(self):
            super().__init__()
            self.quant = QuantStub()
            self.linear = nn.Linear(8, 1)
            self.dequant = DeQuantStub()

        def forward(self, x):
            return self.dequant(torch.sigmoid(self.linear(self.quant(x))))

    m = LogisticRegression()
    m.qconfig = torch.ao.quantization.default_qconfig
    m.train()
    mq = torch.ao.quantization.prepare_qat(m)
    mq.eval()
    mq = torch.ao.quantization.convert(mq)
    ws = float(fields["weight_scale"])
    wq = torch.quantize_per_tensor(torch.tensor(fields["weight"], dtype=torch.float32).reshape(1, 8) * ws,
                                   ws, 0, torch.qint8)
    mq.linear.set_weight_bias(wq, torch.tensor([float(fields["bias"])], dtype=torch.float32))
    mq.linear.scale = float(fields["out_scale"])
    mq.linear.zero_point = int(fields["out_zero_point"])
    mq.quant.scale = torch.tensor([float(fields["in_scale"])])
    mq.quant.zero_point = torch.tensor([int(fields["in_zero_point"])])
    return mq


def score(mq, x: np.ndarray) -> np.ndarray:
    """p (fp32) of every row of x (n x 8 fp32); decision = p > 0.5 (model/model.py:206)."""
    import torch

    with torch.no_grad():
        return mq(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))).numpy().reshape(-1)


def config3_features(n: int, seed: int = 0xF5A3) -> np.ndarray:
    """BASELINE config 3 feature vectors (SURVEY.md §8 d): uniform over the CICIDS input
    ranges (port 0-65535, lengths 0-1500, IATs 0-1.2e8 us), variance = std^2, plus an
    exact grid around the decision boundary acc in [-100, 100] for the first 1/16."""
    rng = np.random.default_rng(seed)
    x = np.empty((n, 8), dtype=np.float32)
    x[:, 0] = rng.integers(0, 65536, n)
    x[:, 1:5] = rng.uniform(0, 1500, (n, 4))
    x[:, 5:8] = rng.uniform(0, 1.2e8, (n, 3))
    x[:, 3] = x[:, 2] ** 2
    m = n // 16   # quantized inputs q = x / 944881.875 in [0, 3]: acc = sum w q near 0
    x[:m] = (rng.integers(0, 4, (m, 8)) * 944881.875).astype(np.float32)
    return x
