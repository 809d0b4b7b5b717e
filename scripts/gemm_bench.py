#!/usr/bin/env python
"""Correlation GEMM at an InLoc volume: the HIP kernels (plain and fused
2x2x2x2 max-pool, bf16 and MX-fp8) against hipBLASLt (torch.mm /
torch._scaled_mm) on the same [M, K] x [N, K]^T problem.

    python scripts/gemm_bench.py [--hw 150 200] [--k 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, nargs=2, default=[150, 200])
    ap.add_argument("--k", type=int, default=1024)
    a = ap.parse_args()
    from ncnet_amd.ops import _ext
    from ncnet_amd.ops.correlation import FP8, FP8_FEAT_SCALE
    C = _ext.ext()
    h, w = a.hw
    M = N = h * w
    K = a.k
    fl = 2.0 * M * N * K
    A = torch.nn.functional.normalize(torch.randn(1, M, K, device="cuda"), dim=-1).to(torch.bfloat16)
    B = torch.nn.functional.normalize(torch.randn(1, N, K, device="cuda"), dim=-1).to(torch.bfloat16)
    out = torch.empty(1, M, N, device="cuda")
    res = {}
    res["hip bf16 plain (fp32 out)"] = timeit(lambda: C.corr_gemm(A, B, out, None, None, 0.0))
    pv = torch.empty(1, h // 2, w // 2, h // 2, w // 2, device="cuda")
    pi = torch.empty(pv.shape, dtype=torch.uint8, device="cuda")
    res["hip bf16 pool2"] = timeit(lambda: C.corr_gemm_pool2(A, B, pv, pi, h, w, h, w, 0.0))
    Ah, Bh = A.half(), B.half()
    res["hip f16 pool2"] = timeit(lambda: C.corr_gemm_pool2(Ah, Bh, pv, pi, h, w, h, w, 0.0))
    A8, B8 = (A.float() * FP8_FEAT_SCALE).to(FP8), (B.float() * FP8_FEAT_SCALE).to(FP8)
    res["hip fp8 plain (fp32 out)"] = timeit(lambda: C.corr_gemm(A8, B8, out, None, None, 1.0 / FP8_FEAT_SCALE ** 2))
    res["hip fp8 pool2"] = timeit(lambda: C.corr_gemm_pool2(A8, B8, pv, pi, h, w, h, w, 1.0 / FP8_FEAT_SCALE ** 2))
    a2, b2 = A[0], B[0]
    res["hipBLASLt bf16 (bf16 out)"] = timeit(lambda: torch.mm(a2, b2.t()))
    try:
        one = torch.ones((), device="cuda")
        res["hipBLASLt fp8 (bf16 out)"] = timeit(lambda: torch._scaled_mm(A8[0], B8[0].t(), one, one,
                                                                        out_dtype=torch.bfloat16))
    except Exception as e:  # noqa: BLE001
        print("scaled_mm unavailable:", repr(e)[:200])
    for k, v in res.items():
        print(f"{k:32s} {v:8.3f} ms  {fl / v / 1e9:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
