"""Host orchestrator — the role of FlowSentryX src/fsx_load.py.

The reference loader (src/fsx_load.py:1-18) was meant to (1) load the data-plane
program, (2) `torch.load` the int8 QAT weights (src/model_weights.pth) and (3) push
them into a BPF map for in-kernel scoring. It never ran (`BPF(text=bpf_program)` is a
NameError at :15 and BCC is absent). This module does the same three things against
libfsx_hip.so: open a context (the program + its five maps), load the weights with a
loader that executes nothing from the file, and hand them to fsx_load_q8_model. It can
also replay a pcap through the data plane in batches.

PyTorch is used here only to read the .pth checkpoint (torch.load(weights_only=True));
the scoring itself runs in libfsx_hip.so.
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import numpy as np

from . import lib


def load_weights(path: str | Path) -> lib.FsxQ8Model:
    """fsx_q8_model from the reference's model_weights.pth (state_dict of the converted
    QuantStub -> Linear(8,1) -> sigmoid -> DeQuantStub, model/model.py:124-137) or from
    its JSON export (tests/golden/model_weights.json)."""
    path = Path(path)
    if path.suffix == ".json":
        d = json.loads(path.read_text())
    else:
        import torch

        sd = torch.load(path, weights_only=True, map_location="cpu")
        w, b = sd["linear._packed_params._packed_params"]
        d = {
            "weight": [int(x) for x in w.int_repr().flatten().tolist()],
            "weight_scale": float(w.q_scale()),
            "bias": float(b.detach().float().flatten()[0]) if b is not None else 0.0,
            "in_scale": float(sd["quant.scale"].flatten()[0]),
            "in_zero_point": int(sd["quant.zero_point"].flatten()[0]),
            "out_scale": float(sd["linear.scale"]),
            "out_zero_point": int(sd["linear.zero_point"]),
        }
    return model_from_dict(d)


def model_from_dict(d: dict) -> lib.FsxQ8Model:
    if len(d["weight"]) != 8:
        raise ValueError("the reference model is Linear(8, 1)")
    m = lib.FsxQ8Model()
    for i, w in enumerate(d["weight"]):
        m.weight[i] = int(w)
    m.weight_scale = float(d["weight_scale"])
    m.bias = float(d["bias"])
    m.in_scale = float(d["in_scale"])
    m.in_zero_point = int(d["in_zero_point"])
    m.out_scale = float(d["out_scale"])
    m.out_zero_point = int(d["out_zero_point"])
    return m


def open_data_plane(weights: str | Path | None = None, **config) -> lib.FsxContext:
    """Open the data plane (fsx() + the five maps of src/fsx_kern.c:56-94) on one GPU and,
    if given, push the model weights into it."""
    ctx = lib.FsxContext(**config)
    if weights is not None:
        ctx.load_q8_model(load_weights(weights))
    return ctx


def replay_pcap(ctx: lib.FsxContext, pcap_path: str | Path, batch: int = 1 << 20):
    """Replay a pcap (ns or µs resolution) through the data plane; yields
    (verdicts, first_index) per batch. Arrival time = the record timestamp."""
    from . import pcap

    start = 0
    for hdr, length, ts in pcap.read_batches(pcap_path, batch):
        yield ctx.verdict_batch(hdr, length, ts), start
        start += len(length)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--weights", default=None, help="model_weights.pth or .json")
    ap.add_argument("--pcap", default=None)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--max-entries", type=int, default=100000)
    args = ap.parse_args(argv)
    ctx = open_data_plane(args.weights, max_entries=args.max_entries, max_batch=args.batch)
    if args.pcap:
        n = d = 0
        for v, _ in replay_pcap(ctx, args.pcap, args.batch):
            n += len(v)
            d += int((v == lib.XDP_DROP).sum())
        a, dr = ctx.stats()
        print(json.dumps({"packets": n, "dropped": d, "stats_map": {"allowed": a, "dropped": dr}}))
    ctx.close()


if __name__ == "__main__":
    main()
