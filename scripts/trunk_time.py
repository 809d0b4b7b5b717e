#!/usr/bin/env python
"""Wall time of the frozen ResNet-101 layer3 trunk plan (FrozenResNetPlan,
bf16, eager) at the InLoc 3200 px size (1 image) and the training size
(32 x 400 px): a quick same-box A/B probe for trunk kernel changes.

    python scripts/trunk_time.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ncnet_amd.models.backbones import FrozenResNetPlan, fold_frozen_bn, resnet_trunk  # noqa: E402


def main():
    torch.manual_seed(0)
    t = resnet_trunk("resnet101", "layer3").eval().cuda()
    plan = FrozenResNetPlan(fold_frozen_bn(t), torch.bfloat16)
    for shape in ((1, 3, 3200, 2400), (32, 3, 400, 400)):
        x = torch.randn(shape, device="cuda")
        with torch.no_grad():
            for _ in range(3):
                plan(x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                plan(x)
            e1.record()
            torch.cuda.synchronize()
        print(f"trunk {tuple(shape)}  {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
