#!/usr/bin/env python
"""Which framework ops launch the small (non-NC) kernels of a training step:
torch.profiler over a few bench.py-equivalent steps, aten ops with their
input shapes and the Python frame that called them, sorted by device time.

    python scripts/step_ops.py [--steps 4] [--top 40] [--out gpurun_out/step_ops.txt]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import DistContext
    dev = torch.device("cuda")
    torch.manual_seed(1)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(dev).train()
    tr = Trainer(m, make_adam([p for p in m.parameters() if p.requires_grad], 5e-4), DistContext(device=dev))
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [{"source_image": torch.randn(16, 3, 400, 400, device=dev, generator=g),
             "target_image": torch.randn(16, 3, 400, 400, device=dev, generator=g)} for _ in range(2)]
    for i in range(3):
        tr.train_step(pool[i % 2], pool[(i + 1) % 2])
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                record_shapes=True, with_stack=True) as prof:
        for i in range(a.steps):
            tr.train_step(pool[i % 2], pool[(i + 1) % 2])
        torch.cuda.synchronize()
    lines = []
    # framework ops (not ncnet kernels) by input shapes: where the small copies come from
    agg = {}
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key.startswith("aten::") and e.device_time_total > 0 and e.key in (
                "aten::cat", "aten::copy_", "aten::sum", "aten::add_", "aten::mul", "aten::clone", "aten::index",
                "aten::to", "aten::_to_copy", "aten::contiguous", "aten::zero_", "aten::fill_", "aten::stack",
                "aten::add", "aten::where", "aten::sub", "aten::div", "aten::mean", "aten::flip", "aten::zeros"):
            agg[(e.key, str(e.input_shapes)[:150])] = (e.device_time_total / a.steps, e.count / a.steps)
    lines.append("per-step device time (us) / calls of framework ops by input shape:")
    for (k, shp), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        lines.append(f"{t:9.1f} us {c:5.1f}x  {k:18s} {shp}")
    t = prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=a.top)
    lines.append(t)
    t2 = prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=a.top)
    lines.append(t2)
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
