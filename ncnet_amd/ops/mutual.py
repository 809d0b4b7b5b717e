"""MutualMatching (lib/model.py:155-175) with a HIP forward and backward.

Forward: one pass of row statistics (max over B for each A cell), one of
column statistics (max over A for each B cell), and an elementwise apply
``c * ((c / (maxA + eps)) * (c / (maxB + eps)))`` in the reference's order.

Backward: ``d/dc`` of ``c^3 / (A B)`` plus the max-routed terms: the row
(column) sum of ``-g * out / A`` (``/ B``) is added to the row's (column's)
argmax element, which is exactly where autograd's ``max(dim)`` backward
routes it.
"""
from __future__ import annotations

import torch

from .. import config as _config
from . import _ext
from . import reference as ref

EPS = ref.MUTUAL_EPS


def _stats(c3: torch.Tensor):
    C = _ext.ext()
    V, R, Cc = c3.shape
    rmax = torch.empty((V, R), dtype=torch.float32, device=c3.device)
    rarg = torch.empty((V, R), dtype=torch.int32, device=c3.device)
    cmax = torch.empty((V, Cc), dtype=torch.float32, device=c3.device)
    carg = torch.empty((V, Cc), dtype=torch.int32, device=c3.device)
    # both maxima in one pass over the volume (stats2d) when rows are 16-byte multiples
    if not (_config.RUNTIME.stats2d and C.stats2d(c3, rmax, rarg, None, cmax, carg, None, 0)):
        C.stats_rows(c3, rmax, rarg, None, 0)
        C.stats_cols(c3, cmax, carg, None, 0)
    return rmax, rarg, cmax, carg


class MutualMatchingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, corr4d, pad_ks: int = 0):
        V, ch, I, J, K, L = corr4d.shape
        assert ch == 1
        c3 = corr4d.reshape(V, I * J, K * L).float().contiguous()
        rmax, rarg, cmax, carg = _stats(c3)
        out = torch.empty_like(c3)
        xp = None
        if pad_ks:
            # the padded bf16 NC-input planes of both symmetric branches in the same
            # pass (csrc/volume.hip mm_apply PAD mode, halos included)
            _, ppl = _ext.ext().pad_geom(K, L, pad_ks)
            xp = torch.empty((2 * V * I * J, ppl), dtype=torch.bfloat16, device=c3.device)
            _ext.ext().mm_apply(c3, rmax, cmax, out, xp[:V * I * J], xp[V * I * J:], EPS, [pad_ks, I, J])
            ctx.mark_non_differentiable(xp)
        else:
            _ext.ext().mm_apply(c3, rmax, cmax, out, None, None, EPS)
        ctx.save_for_backward(c3, rmax, rarg, cmax, carg)
        ctx.shape = corr4d.shape
        if xp is not None:
            return out.reshape(corr4d.shape), xp
        return out.reshape(corr4d.shape)

    @staticmethod
    def backward(ctx, g, *_):
        c3, rmax, rarg, cmax, carg = ctx.saved_tensors
        g3 = g.reshape(c3.shape).float().contiguous()
        gc = torch.empty_like(c3)
        _ext.ext().mm_bwd(c3, g3, rmax, rarg, cmax, carg, gc, EPS, _config.RUNTIME.stats2d)   # one pass for both sums
        return gc.reshape(ctx.shape), None


def mutual_matching_padded(corr4d: torch.Tensor, ks: int):
    """MutualMatching (autograd) that also writes its output as the zero-padded
    bf16 planes of both symmetric NeighConsensus branches for a first layer of
    kernel size ``ks`` (the training stack's conv1x16 / wgrad1x16 operand,
    ops/neigh_consensus.py fast1x path) -> (x [V,1,I,J,K,L] fp32, planes
    [2 V I J, PPL] bf16).  Square volumes only."""
    V, ch, I, J, K, L = corr4d.shape
    assert ch == 1 and (I, J) == (K, L)
    return MutualMatchingFn.apply(corr4d, ks)


def mutual_matching_nc_input(corr4d: torch.Tensor, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """Inference MutualMatching written straight as the bf16 input of both
    symmetric NeighConsensus branches: [2V, I, J, K, L] with x in the first V
    volumes and its A<->B swap in the last V (mm_apply's bf16 and transposed
    bf16 outputs; no fp32 volume, no cast, no separate transpose).  Square
    volumes only (I, J) == (K, L).  ``dtype``: bf16, or float16 (half_precision models)."""
    V, ch, I, J, K, L = corr4d.shape
    assert ch == 1 and (I, J) == (K, L)
    c3 = corr4d.reshape(V, I * J, K * L).float().contiguous()
    rmax, _, cmax, _ = _stats(c3)
    x2 = torch.empty((2 * V, I, J, K, L), dtype=dtype, device=c3.device)
    _ext.ext().mm_apply(c3, rmax, cmax, None, x2[:V].view(V, I * J, K * L), x2[V:].view(V, K * L, I * J), EPS)
    return x2


def mutual_matching(corr4d: torch.Tensor) -> torch.Tensor:
    if _ext.use_hip(corr4d):
        return MutualMatchingFn.apply(corr4d)
    return ref.mutual_matching(corr4d)
