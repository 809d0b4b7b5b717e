#!/usr/bin/env python
"""ResNet stem (7x7/2 conv, Cin = 3, + bias + ReLU + 3x3/2 max-pool) at the
InLoc 3200 px and 400 px training shapes: MIOpen's direct bf16 convolution
(the FrozenResNetPlan path before round 5's native stem, solver picked with
cudnn.benchmark on and off) against the native stem -- HIP im2col
(csrc/epilogue.hip stem_im2col16) + one K = 192 GEMM (native conv2d_nhwc as a
1x1, or hipBLASLt) -- each followed by the fused bias / ReLU / max-pool
kernel.  Prints one JSON line per (shape, variant) with the time and the max
error against an fp32 reference of the same bf16 operands.

    python scripts/stem_bench.py [--out gpurun_out/stem_bench.jsonl]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ncnet_amd.ops import _ext  # noqa: E402


def timeit(fn, reps=10):
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
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda")
    cl = torch.channels_last
    torch.manual_seed(0)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
    b = torch.randn(64, device=dev) * 0.1
    KP = 192
    wk = w.permute(0, 2, 3, 1).reshape(64, 147)
    wk = torch.cat((wk, wk.new_zeros(64, KP - 147)), 1).contiguous()   # [64, KP] bf16
    w11 = wk.view(64, KP, 1, 1).contiguous(memory_format=cl)
    wt = wk.t().contiguous()
    zb = torch.zeros(64, device=dev)
    recs = []
    for name, n, H, W in (("inloc_3200", 1, 2400, 3200), ("train_400_chunk32", 32, 400, 400)):
        x = torch.randn(n, 3, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
        Hp, Wp = (Ho + 2 - 3) // 2 + 1, (Wo + 2 - 3) // 2 + 1
        out = torch.empty(n, 64, Hp, Wp, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        ref = F.max_pool2d(F.relu(F.conv2d(x.float(), w.float(), b, 2, 3)), 3, 2, 1)
        A = torch.empty(n * Ho * Wo, KP, device=dev, dtype=torch.bfloat16)
        y = torch.empty(n, 64, Ho, Wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)

        def miopen():
            yy = F.conv2d(x, w, None, 2, 3).contiguous(memory_format=cl)
            C.maxpool_bias_act(yy, b, out, 3, 2, 1, 1)

        def native():
            C.stem_im2col16(x, A, 7, 7, 2, 3)
            C.conv2d_nhwc(A.view(n, Ho, Wo, KP).permute(0, 3, 1, 2), w11, zb, None, y, 1, 0, 0)
            C.maxpool_bias_act(y, b, out, 3, 2, 1, 1)

        def blas():
            C.stem_im2col16(x, A, 7, 7, 2, 3)
            yy = torch.mm(A, wt).view(n, Ho, Wo, 64).permute(0, 3, 1, 2)
            C.maxpool_bias_act(yy, b, out, 3, 2, 1, 1)

        def im2col_only():
            C.stem_im2col16(x, A, 7, 7, 2, 3)

        for bm in (True, False):
            torch.backends.cudnn.benchmark = bm
            for vname, fn in (("miopen", miopen), ("native", native), ("blas", blas), ("im2col_only", im2col_only)):
                if vname != "miopen" and not bm:
                    continue
                t = timeit(fn)
                err = None
                if vname != "im2col_only":
                    fn()
                    torch.cuda.synchronize()
                    err = float((out.float() - ref).abs().max() / ref.abs().max())
                r = {"shape": name, "variant": vname, "cudnn_benchmark": bm, "ms": round(t, 4), "rel_max_err": err}
                print(json.dumps(r), flush=True)
                recs.append(r)
        del A, y, x, out, ref
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
