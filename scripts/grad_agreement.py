#!/usr/bin/env python
"""First-step NC gradient agreement at the training-quality operating point.

Same init and batch; gradients of the weak loss w.r.t. every NC parameter from
(1) the HIP training path (``--nc-precision bf16`` default), (2) the fp32
reference algorithm, (3) the reference algorithm under bf16 autocast.  Prints
loss values, gradient norms and cosine similarities per parameter.

    python scripts/grad_agreement.py --image-size 240
"""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.data.datasets import synthetic_correspondence_batch  # noqa: E402
from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_weak_loss  # noqa: E402
from ncnet_amd.engine.trainer import weak_loss  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402
from train_quality import recalibrate_bn  # noqa: E402


def grads(model):
    return [p.grad.detach().double().clone() for p in model.NeighConsensus.parameters()]


def cos(a, b):
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-300))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--image-size", type=int, default=240)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--last-layer", type=str, default="", help="trunk cut (default layer3, the reference's)")
    ap.add_argument("--bias", type=float, default=0.05)
    a = ap.parse_args(argv)
    dev = torch.device("cuda")
    torch.manual_seed(a.seed)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1],
                   feature_extraction_last_layer=a.last_layer).to(dev)
    recalibrate_bn(m, a.image_size, dev)
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, a.bias)
    b = synthetic_correspondence_batch(a.batch, a.image_size, dev, seed=0)
    b = {"source_image": b["source_image"], "target_image": b["target_image"]}
    out = {}
    copies = {"ref32": copy.deepcopy(m), "ref16": copy.deepcopy(m)}   # before the trunk plan holds a HIP graph
    m.train()
    loss = weak_loss(m, b)
    loss.backward()
    g_h = grads(m)
    out["loss_hip"] = float(loss.detach())
    res = {}
    for name, dt in (("ref32", torch.float32), ("ref16", torch.bfloat16)):
        mr = copies[name]
        for p in mr.parameters():
            p.grad = None
        mr.train()
        lr = reference_weak_loss(ReferenceAlgorithm(mr, dt), b)
        lr.backward()
        res[name] = grads(mr)
        out[f"loss_{name}"] = float(lr.detach())
    names = [n for n, _ in m.NeighConsensus.named_parameters()]
    for i, n in enumerate(names):
        out[n] = {"norm_hip": float(g_h[i].norm()), "norm_ref32": float(res["ref32"][i].norm()),
                  "cos_hip_ref32": cos(g_h[i], res["ref32"][i]), "cos_ref16_ref32": cos(res["ref16"][i], res["ref32"][i]),
                  "cos_hip_ref16": cos(g_h[i], res["ref16"][i])}
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    main()
