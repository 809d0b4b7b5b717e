#!/usr/bin/env python
"""Probe: does the InLoc PairMatcher graph capture survive the bench process
state (headline training steps with cudnn.benchmark=True first)?  Prints the
full traceback of a failed capture so the offending call is named.

    python scripts/probe/pair_graph_probe.py --train-steps 3 --size 1600
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=3)
    ap.add_argument("--size", type=int, default=1600)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    from ncnet_amd.models import ImMatchNet
    if a.train_steps:
        from ncnet_amd.engine.trainer import Trainer, make_adam
        from ncnet_amd.parallel.dist import DistContext
        m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(dev).train()
        params = [p for p in m.parameters() if p.requires_grad]
        tr = Trainer(m, make_adam(params, 5e-4), DistContext(device=dev))
        pool = [{"source_image": torch.randn(16, 3, 400, 400, device=dev),
                 "target_image": torch.randn(16, 3, 400, 400, device=dev)} for _ in range(2)]
        for i in range(a.train_steps):
            tr.train_step(pool[i % 2], pool[(i + 1) % 2])
        torch.cuda.synchronize()
        print("trained", a.train_steps, flush=True)
    from ncnet_amd.eval import inloc
    made = []
    orig = inloc.PairMatcher.__init__

    def init(self, *args, **kw):
        orig(self, *args, **kw)
        made.append(self)
    inloc.PairMatcher.__init__ = init
    import bench
    sec = bench._inloc_secondary()
    print(json.dumps(sec), flush=True)
    for pm in made:
        if pm.capture_error:
            print(pm.capture_error, flush=True)
            break

if __name__ == "__main__":
    main()
