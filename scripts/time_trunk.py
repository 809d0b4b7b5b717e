#!/usr/bin/env python
"""Time the frozen trunk alone (HIP events, back-to-back calls, no host syncs
in between) at a given image size: separates GPU time from launch gaps."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ncnet_amd.models import ImMatchNet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, nargs=2, default=[2400, 3200])
ap.add_argument("--batch", type=int, default=2)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--chunk", type=int, nargs="+", default=[0], help="run the batch in chunks of this many images "
                "(0: whole batch); several values are timed in turn")
a = ap.parse_args()
m = ImMatchNet(use_cuda=True, ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1]).cuda().eval()
x = torch.randn(a.batch, 3, *a.hw, device="cuda")


def run(chunk):
    if not chunk or chunk >= a.batch:
        return m.FeatureExtraction.trunk_forward(x, torch.bfloat16)
    return torch.cat([m.FeatureExtraction.trunk_forward(x[c:c + chunk], torch.bfloat16)
                      for c in range(0, a.batch, chunk)])


gflop = 44.6 * (a.hw[0] * a.hw[1]) / (400 * 400) * a.batch
with torch.inference_mode():
    for chunk in a.chunk:
        for _ in range(3):
            f = run(chunk)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(a.iters):
            f = run(chunk)
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / a.iters
        print(f"trunk {a.batch}x{a.hw} chunk {chunk}: {e0.elapsed_time(e1) / a.iters:.3f} ms GPU, {wall:.3f} ms wall, "
              f"{gflop / (e0.elapsed_time(e1) / a.iters) :.1f} TFLOP/s, out {tuple(f.shape)}", flush=True)
