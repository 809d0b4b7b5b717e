"""The HIP training path's math in float64, rounded to bf16 exactly where the
kernels store bf16 -- a tight end-to-end oracle for gradient tests.

The fused path (models/immatchnet.py ``weak_loss_volumes``) stores bf16 at:
the L2-normalised features (GEMM operands), the NeighConsensus input
(MutualMatching output), every hidden NC activation, the packed NC weights,
and -- in backward -- the gradient w.r.t. every NC layer's pre-activation
(after its ReLU mask).  Everything else (correlation and conv accumulation,
MutualMatching, the symmetric combine, the weak loss, the gradients below the
NC input) is fp32 there and fp64 here.  With those roundings reproduced, the
only differences left are fp32-vs-fp64 accumulation order and the rare
element whose rounding lands on the other side of a bf16 boundary, so
gradients agree to ~1e-3 instead of the ~10-20 % that separate bf16 from an
unrounded fp32 reference (tests/test_gpu_quality.py).

Semantics follow the reference: lib/model.py:14-17 (L2 norm), 106-115
(correlation), 155-175 (MutualMatching), 122-153 (symmetric NC),
lib/conv4d.py:11-51 (Conv4d), train.py:110-156 (weak loss, rolled negatives).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import reference as ref


def q(x: torch.Tensor) -> torch.Tensor:
    """Forward bf16 rounding, straight-through gradient."""
    return x + (x.to(torch.bfloat16).to(x.dtype) - x).detach()


class _QGrad(torch.autograd.Function):
    """Identity forward; the incoming gradient is rounded to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def qgrad(x: torch.Tensor) -> torch.Tensor:
    return _QGrad.apply(x)


def nc_stack(x: torch.Tensor, ws_std, bs) -> torch.Tensor:
    """One NC branch: x [V,1,I,J,K,L] (already bf16-valued) -> last ReLU output."""
    h = x
    n = len(ws_std)
    for li, (w, b) in enumerate(zip(ws_std, bs)):
        pre = ref.conv4d(h, ref.conv4d_weight_from_std(q(w))) + b.view(1, -1, 1, 1, 1, 1)
        act = torch.relu(qgrad(pre))
        h = act if li == n - 1 else q(act)
    return h


def neigh_consensus(x: torch.Tensor, ws_std, bs, symmetric: bool = True) -> torch.Tensor:
    xq = q(x)
    y = nc_stack(xq, ws_std, bs)
    if symmetric:
        y = y + ref.swap_ab(nc_stack(ref.swap_ab(xq), ws_std, bs))
    return y


def weak_loss_volumes(feats: torch.Tensor, hw, b: int, ws_std, bs, normalize: bool = True,
                      dtype=torch.float64) -> torch.Tensor:
    """feats: [2b, C, h, w] raw trunk features (normalize=True) or the packed
    L2-normalised rows [2b, h*w, C] (normalize=False).  Returns the [2b,1,h,w,h,w]
    positive + rolled-negative volumes of the weak loss (train.py:121,137-138)."""
    h, w = hw
    if normalize:
        f = ref.feature_l2norm(feats.to(dtype))
        f = f.reshape(f.shape[0], f.shape[1], h * w).transpose(1, 2)
    else:
        f = feats.to(dtype)
    f = q(f)
    fa, fb = f[:b], f[b:]
    roll = torch.as_tensor(np.roll(np.arange(b), -1), device=f.device)
    A = torch.cat((fa, fa[roll]))
    B = torch.cat((fb, fb))
    corr = torch.bmm(A, B.transpose(1, 2)).view(2 * b, 1, h, w, h, w)
    corr = ref.mutual_matching(corr)
    corr = neigh_consensus(corr, [w_.to(dtype) for w_ in ws_std], [b_.to(dtype) for b_ in bs])
    return ref.mutual_matching(corr)
