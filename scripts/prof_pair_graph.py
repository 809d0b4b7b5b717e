#!/usr/bin/env python
"""Replay the InLoc pair graph (eval/inloc.py PairMatcher: correlation + pool,
MutualMatching, fused NC, MutualMatching, match extraction) on fixed features
W + N times, for a per-pair kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pg -o run -- \
        python3 scripts/prof_pair_graph.py --image-size 3200 --pairs 10
    python3 scripts/prof_summary.py <trace> --marker corr_gemm --warmup 3 --steps 10
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd.eval.inloc import PairMatcher  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image-size", type=int, default=3200)
    ap.add_argument("--pairs", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], dtype="bf16", relocalization_k_size=2).to(dev).eval()
    h, w = a.image_size * 3 // 4, a.image_size
    img = torch.randn(2, 3, h, w, device=dev)
    with torch.inference_mode():
        f, (fh, fw) = model.extract(img)
        fa, fb = f[:1], f[1:]
        matcher = PairMatcher(model, 2)
        for _ in range(a.warmup + a.pairs):
            res, cnt = matcher(fa, (fh, fw), fb, (fh, fw))
        torch.cuda.synchronize()
    print(f"graphed={matcher.graphed} matches={int(cnt)}")


if __name__ == "__main__":
    main()
