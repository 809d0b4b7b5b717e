#!/usr/bin/env python
"""Per-layer trunk conv microbenchmark: the native NHWC implicit-GEMM kernel
(csrc/conv2d.hip) vs hipBLASLt (1x1 convs as GEMMs, bias+ReLU epilogue) and
MIOpen (F.conv2d, channels-last bf16) at the ResNet-101 layer shapes of the
InLoc 3200 px trunk (2 images) or the 400 px training trunk (32 images).

    python scripts/conv_bench.py [--res 3200|400]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ncnet_amd.ops import _ext  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=3200)
    ap.add_argument("--n", type=int, default=0, help="images (default: 2 at 3200 px, 32 at 400 px)")
    ap.add_argument("--residual", action="store_true",
                    help="the n3 layers with their bottleneck residual (as the trunk runs them); auto variant only")
    a = ap.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda")
    cl = torch.channels_last
    if a.res == 3200:
        n, hw = 2, {1: (600, 800), 2: (300, 400), 3: (150, 200)}
    else:
        n, hw = 32, {1: (100, 100), 2: (50, 50), 3: (25, 25)}
    n = a.n or n
    # (name, layer, cin, cout, k, stride, input hw layer)
    shapes = [("l1.nd", 1, 64, 256, 1, 1, 1), ("l1.n1", 1, 256, 64, 1, 1, 1), ("l1.n2", 1, 64, 64, 3, 1, 1), ("l1.n3", 1, 64, 256, 1, 1, 1),
              ("l2.n1", 2, 512, 128, 1, 1, 2), ("l2.n2", 2, 128, 128, 3, 1, 2), ("l2.n3", 2, 128, 512, 1, 1, 2),
              ("l3.n1", 3, 1024, 256, 1, 1, 3), ("l3.n2", 3, 256, 256, 3, 1, 3), ("l3.n3", 3, 256, 1024, 1, 1, 3),
              ("l3.nd", 3, 512, 1024, 1, 2, 2), ("l3.n2s", 3, 256, 256, 3, 2, 2)]
    print(f"{'layer':8s} {'M':>8s} {'N':>5s} {'K':>5s}  {'native v1':>16s}  {'native v2':>16s}"
          f"  {'v3 (chip round)':>16s}  {'auto':>16s}  {'hipBLASLt/MIOpen':>18s}")
    for name, _, cin, cout, k, s, lin in shapes:
        H, W = hw[lin]
        x = torch.randn(n, cin, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        b = torch.randn(cout, device=dev)
        Ho, Wo = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
        y = torch.empty(n, cout, Ho, Wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        M, K = n * Ho * Wo, cin * k * k
        fl = 2.0 * M * cout * K
        res = None
        if a.residual and name.endswith(".n3"):
            res = torch.randn_like(y)
        run = lambda: C.conv2d_nhwc(x, w, b, res, y, s, k // 2, 1)   # noqa: E731
        if a.residual:
            # every 1x1 stride-1 conv as the trunk runs it (n3 with its residual):
            # the native kernel vs hipBLASLt with the same fused epilogue
            # (csrc/gemm_lt.hip, candidates timed once) -- models/backbones.py
            # 'auto' takes the faster per shape
            if not (k == 1 and s == 1):
                continue
            C.set_tuning("conv2d_variant", 0)
            t_a = timeit(run)
            C.gemm_lt(x, w, b, res, y, 1, 1)
            t_l = timeit(lambda: C.gemm_lt(x, w, b, res, y, 1, 0))
            gb = (x.numel() + (2 if res is not None else 1) * y.numel()) * 2 / 1e9
            tag = "+res" if res is not None else "    "
            print(f"{name:8s}{tag} M={M} N={cout} K={K}: native {t_a * 1e3:7.1f} us {fl / t_a / 1e9:5.0f} TF "
                  f"{gb / t_a * 1e3:5.2f} TB/s | hipBLASLt {t_l * 1e3:7.1f} us {fl / t_l / 1e9:5.0f} TF "
                  f"{gb / t_l * 1e3:5.2f} TB/s | auto {min(t_a, t_l) * 1e3:7.1f} us", flush=True)
            continue
        C.set_tuning("conv2d_variant", 1)
        t_1 = timeit(run)
        C.set_tuning("conv2d_variant", 2)
        t_n = timeit(run)
        C.set_tuning("conv2d_variant", 3)
        t_3 = timeit(run)
        C.set_tuning("conv2d_variant", 0)
        t_a = timeit(run)
        if k == 1 and s == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
            w2 = w.reshape(cout, cin)
            bb = b.to(torch.bfloat16)
            t_o = timeit(lambda: torch._addmm_activation(bb, x2, w2.t()))
        else:
            wb = w
            t_o = timeit(lambda: torch.relu_(torch.nn.functional.conv2d(x, wb, b.to(torch.bfloat16), s, k // 2)))
        print(f"{name:8s} {M:8d} {cout:5d} {K:5d}  {t_1 * 1e3:7.1f} us {fl / t_1 / 1e9:5.0f} TF  "
              f"{t_n * 1e3:7.1f} us {fl / t_n / 1e9:5.0f} TF  "
              f"{t_3 * 1e3:7.1f} us {fl / t_3 / 1e9:5.0f} TF  {t_a * 1e3:7.1f} us {fl / t_a / 1e9:5.0f} TF  "
              f"{t_o * 1e3:7.1f} us {fl / t_o / 1e9:5.0f} TF", flush=True)


if __name__ == "__main__":
    main()
