#!/usr/bin/env python
"""Correlation GEMM at the InLoc 3200 px shape (150 x 200 features per image,
1024 channels, k = 2 fused 2x2x2x2 max-pool): bf16 vs MX-fp8 operands, and
hipBLASLt's plain GEMM (no pool) as the rate reference.

    python scripts/corr_bench.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, reps):
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
    from ncnet_amd.ops.correlation import correlation_pool2, l2norm_pack, l2norm_pack_fp8
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    h, w, c = 150, 200, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    cl = torch.channels_last     # the trunk's output layout and dtype
    fa = torch.randn(1, c, h, w, device=dev, generator=g).relu().to(torch.bfloat16).contiguous(memory_format=cl)
    fb = torch.randn(1, c, h, w, device=dev, generator=g).relu().to(torch.bfloat16).contiguous(memory_format=cl)
    flop = 2.0 * (h * w) ** 2 * c
    out = {}
    pa, pb = l2norm_pack(fa), l2norm_pack(fb)
    out["bf16_pool"] = timeit(lambda: correlation_pool2(pa, pb, h, w, h, w, packed=True), a.reps)
    qa, qb = l2norm_pack_fp8(fa), l2norm_pack_fp8(fb)
    out["fp8_pool"] = timeit(lambda: correlation_pool2(qa, qb, h, w, h, w, packed=True), a.reps)
    A = pa.reshape(h * w, c)
    B = pb.reshape(h * w, c)
    out["hipblaslt_bf16_nopool"] = timeit(lambda: torch.matmul(A, B.t()), a.reps)
    for k, ms in out.items():
        print(json.dumps({"case": k, "ms": round(ms, 3), "tflops": round(flop / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
