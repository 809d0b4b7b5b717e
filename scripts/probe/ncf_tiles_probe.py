"""Fused InLoc NC (csrc/nc_fused.hip) at the 3200 px volume [2, 75, 100, 75,
100]: time the kernel for several (R planes per workgroup, IR rows per
workgroup) choices, incl. the one-16-wave-workgroup-per-CU variant (LDS > 80
KB), on one box, interleaved.  Diagnostic for ops/neigh_consensus.py
fused_tiles."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from ncnet_amd.ops import _ext  # noqa: E402
from ncnet_amd.ops import reference as ref  # noqa: E402

nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(5)
x2 = torch.rand((2, 75, 100, 75, 100), device=dev, generator=g).to(torch.bfloat16)
ws = [ref.conv4d_weight_from_std(torch.randn(16, 1, 3, 3, 3, 3, device=dev, generator=g) * 0.2),
      ref.conv4d_weight_from_std(torch.randn(1, 16, 3, 3, 3, 3, device=dev, generator=g) * 0.1)]
bs = [torch.rand(16, device=dev, generator=g) * 0.1, torch.rand(1, device=dev, generator=g) * 0.1]
wts = nc._fused_weights(ws, bs)
y = torch.empty((2, 75, 100, 75, 100), device=dev)
print("fused_tiles ->", nc.fused_tiles(2, 75, 100, 75, 100), flush=True)
cfgs = [(10, 75), (20, 75), (20, 37), (8, 75), (10, 37), (25, 75)]
C = _ext.ext()
ref_y = None
for rnd in range(3):
    for (R, IR) in cfgs:
        fn = lambda: C.nc_fused_k3(x2, *wts, y, R, IR, 15, 20)
        fn()
        torch.cuda.synchronize()
        if rnd == 0:
            if ref_y is None:
                ref_y = y.clone()
            assert torch.equal(y, ref_y) or (y - ref_y).abs().max() < 1e-3, (R, IR)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"round {rnd} R={R:3d} IR={IR:3d}: {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)
