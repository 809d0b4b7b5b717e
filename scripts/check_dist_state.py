"""Pre-flight for the multi-GPU bench: every tensor that broadcast_module
sends over RCCL must live on the rank's GPU (RCCL rejects host tensors),
and the gradient bucket must cover exactly the trainable parameters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.parallel.dist import GradBucket, init_distributed  # noqa: E402

ctx = init_distributed()
m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(ctx.device)
bad = [k for k, v in m.state_dict().items() if v.device != ctx.device]
params = [p for p in m.parameters() if p.requires_grad]
b = GradBucket(params, ctx)
print({"device": str(ctx.device), "state_tensors": len(m.state_dict()), "off_device": bad,
       "bucket_numel": b.flat.numel(), "trainable": sum(p.numel() for p in params)})
assert not bad, bad
