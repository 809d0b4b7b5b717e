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


def _rl2(a, b) -> float:
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def training_grad_errors(fe_finetune: int = 0, point_seed: int = 0, batch_seed: int = 7,
                         device: str = "cuda") -> dict:
    """Relative L2 errors of the fused training path against this oracle at a
    non-degenerate operating point (tests/test_gpu_quality.py,
    scripts/oracle_tolerance.py): a 5,5,5 / 16,16,1 model after three NC Adam
    steps on known-correspondence pairs (trunk frozen, seeds ``point_seed`` ..
    +2), then one weak-loss-volume backward with a random cotangent on batch
    ``batch_seed``.  Keys: 'vols', 'nc0' .. 'nc5' (weight, bias per layer),
    'layer0' .. 'layer2' (each layer's weight and bias gradients as one vector) and,
    with ``fe_finetune`` (the last layer3 bottleneck unfrozen, train.py:60-63),
    'd_raw_features' (the gradient w.r.t. the raw trunk features)."""
    from ..data.datasets import synthetic_correspondence_batch
    from ..engine.trainer import make_adam, weak_loss
    from ..models import ImMatchNet
    from ..ops.correlation import l2norm_pack
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(device)
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.05)
    m.train()
    opt = make_adam([p for p in m.parameters() if p.requires_grad], 5e-4)
    for s in range(3):
        b = synthetic_correspondence_batch(2, 240, device, seed=point_seed + s)
        opt.zero_grad(set_to_none=True)
        weak_loss(m, {"source_image": b["source_image"], "target_image": b["target_image"]}).backward()
        opt.step()
    if fe_finetune:
        for p in m.FeatureExtraction.model[-1][-1].parameters():
            p.requires_grad = True
    b = synthetic_correspondence_batch(2, 240, device, seed=batch_seed)
    imgs = torch.cat((b["source_image"], b["target_image"]))
    opt.zero_grad(set_to_none=True)
    if fe_finetune:
        raw = m.FeatureExtraction.trunk_forward(imgs, torch.bfloat16).detach().requires_grad_(True)
        f, hw = l2norm_pack(raw), tuple(raw.shape[-2:])
    else:
        with torch.no_grad():
            f, hw = m.extract(imgs)
    vols = m.weak_loss_volumes_from_features(f, hw, 2)
    gen = torch.Generator(device=vols.device).manual_seed(batch_seed)
    G = torch.randn(vols.shape, device=vols.device, dtype=vols.dtype, generator=gen)
    (vols * G).sum().backward()
    g_hip = [p.grad.detach().double().clone() for p in m.NeighConsensus.parameters()]
    layers = m.NeighConsensus.conv_layers()
    ws = [ref.conv4d_weight_to_std(l.weight_ref()).detach().double().requires_grad_(True) for l in layers]
    bs = [l.bias.detach().double().requires_grad_(True) for l in layers]
    if fe_finetune:
        raw64 = raw.detach().double().requires_grad_(True)
        ovols = weak_loss_volumes(raw64, hw, 2, ws, bs, normalize=True)
    else:
        ovols = weak_loss_volumes(f.detach(), hw, 2, ws, bs, normalize=False)
    (ovols * G.double()).sum().backward()
    errs = {"vols": _rl2(vols, ovols)}
    o_grads = []
    for w, x in zip(ws, bs):
        o_grads += [w.grad, x.grad]
    flat_h, flat_o = [], []
    for i, (gh, go) in enumerate(zip(g_hip, o_grads)):
        if gh.dim() == 6:
            go = ref.conv4d_weight_from_std(go)
        errs[f"nc{i}"] = _rl2(gh, go)
        flat_h.append(gh.reshape(-1)); flat_o.append(go.reshape(-1))
    # per layer, weight and bias gradients as one vector: the Cout = 1 layer's
    # bias gradient is a single sum over all voxels whose relative error alone
    # is ill-conditioned wherever that sum cancels
    for li in range(len(layers)):
        errs[f"layer{li}"] = _rl2(torch.cat(flat_h[2 * li:2 * li + 2]), torch.cat(flat_o[2 * li:2 * li + 2]))
    if fe_finetune:
        errs["d_raw_features"] = _rl2(raw.grad, raw64.grad)
    return errs
