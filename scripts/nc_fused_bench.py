#!/usr/bin/env python
"""Timing of the fused InLoc NC kernel (csrc/nc_fused.hip) and of the
layer-by-layer path it replaces, at an InLoc volume; optional tiling sweep.

    python scripts/nc_fused_bench.py [--dims 75 100 75 100] [--vols 2] [--sweep "R,IR,TK,TL;..."]
"""
import argparse
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd.ops import _ext  # noqa: E402
nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
from ncnet_amd.ops import reference as ref  # noqa: E402


def timeit(fn, reps):
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
    ap.add_argument("--dims", type=int, nargs=4, default=[75, 100, 75, 100])
    ap.add_argument("--vols", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sweep", type=str, default="")
    ap.add_argument("--layerwise", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    I, J, K, L = a.dims
    x0 = torch.rand(a.vols, I, J, K, L, device=dev).to(torch.bfloat16)
    w1 = ref.conv4d_weight_from_std(torch.randn(16, 1, 3, 3, 3, 3, device=dev) * 0.1)
    w2 = ref.conv4d_weight_from_std(torch.randn(1, 16, 3, 3, 3, 3, device=dev) * 0.05)
    b1, b2 = torch.rand(16, device=dev) * 0.1, torch.full((1,), 0.05, device=dev)
    wts = nc._fused_weights([w1, w2], [b1, b2])
    y = torch.empty(x0.shape, device=dev)
    auto = nc.fused_tiles(a.vols, I, J, K, L)
    cfgs = [auto] + [tuple(int(v) for v in c.split(",")) for c in a.sweep.split(";") if c]
    for R, IR, TK, TL in [(c[2], c[3], c[0], c[1]) for c in cfgs[:1]] + [c for c in cfgs[1:]]:
        ms = timeit(lambda: _ext.ext().nc_fused_k3(x0, *wts, y, R, IR, TK, TL), a.reps)
        print(f"fused R={R:3d} IR={IR:3d} TK={TK:3d} TL={TL:3d}: {ms:8.3f} ms", flush=True)
    if a.layerwise:
        x = x0.float().reshape(a.vols, 1, I, J, K, L)
        nc.FUSED = False
        with torch.inference_mode():
            ms = timeit(lambda: nc.neigh_consensus(x, [w1, w2], [b1, b2], [16, 1], symmetric=False), a.reps)
        print(f"layerwise (ij) non-symmetric: {ms:8.3f} ms")


if __name__ == "__main__":
    main()
