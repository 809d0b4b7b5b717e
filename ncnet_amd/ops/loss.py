"""Weak-supervision score (train.py:110-156) with a fused HIP forward/backward.

For the default ``'softmax'`` normalisation, ``max_j softmax(x)_j =
1 / sum_j exp(x_j - max x)``: the forward needs only the online-softmax row /
column statistics and the backward has the closed form
``ds/dx_j = s (delta_{j, argmax} - softmax_j)``.  ``None`` and ``'l1'``
normalisations use the PyTorch oracle path.
"""
from __future__ import annotations

import torch

from . import _ext
from . import reference as ref


def _row_col_stats(x3: torch.Tensor):
    C = _ext.ext()
    V, R, Cc = x3.shape
    f = dict(dtype=torch.float32, device=x3.device)
    rmax, rse = torch.empty((V, R), **f), torch.empty((V, R), **f)
    cmax, cse = torch.empty((V, Cc), **f), torch.empty((V, Cc), **f)
    rarg = torch.empty((V, R), dtype=torch.int32, device=x3.device)
    carg = torch.empty((V, Cc), dtype=torch.int32, device=x3.device)
    C.stats_rows(x3, rmax, rarg, rse)
    C.stats_cols(x3, cmax, carg, cse)
    return rmax, rarg, rse, cmax, carg, cse


class SoftmaxMaxScoreFn(torch.autograd.Function):
    """sum_v wr[v] * sum_rows s_row + wc[v] * sum_cols s_col (s = max softmax)."""

    @staticmethod
    def forward(ctx, x3, wr, wc):
        x3 = x3.float().contiguous()
        st = _row_col_stats(x3)
        rmax, rarg, rse, cmax, carg, cse = st
        val = (wr.view(-1, 1) / rse).sum() + (wc.view(-1, 1) / cse).sum()
        ctx.save_for_backward(x3, wr, wc, *st)
        return val

    @staticmethod
    def backward(ctx, g):
        x3, wr, wc, rmax, rarg, rse, cmax, carg, cse = ctx.saved_tensors
        gx = torch.empty_like(x3)
        _ext.ext().softmax_max_bwd(x3, rmax, rarg, rse, cmax, carg, cse, wr.float().contiguous(),
                                   wc.float().contiguous(), gx)
        return gx * g, None, None


_WEIGHTS: dict = {}


def _loss_weights(b: int, R: int, Cc: int, device):
    """Per-volume weights of score_neg - score_pos: -1/(2bR), -1/(2bCc) for the
    b positive volumes, + for the b negatives.  Built on the device by fill
    kernels (no pageable host->device copy per step) and cached per shape."""
    key = (b, R, Cc, str(device))
    w = _WEIGHTS.get(key)
    if w is None:
        sign = torch.ones(2 * b, dtype=torch.float32, device=device)
        sign[:b] = -1.0
        w = (sign / (2.0 * b * R), sign / (2.0 * b * Cc))
        if not (sign.is_cuda and torch.cuda.is_current_stream_capturing()):
            _WEIGHTS[key] = w
    return w


def weak_loss_from_corr(corr4d: torch.Tensor, n_pos: int, normalization: str | None = "softmax") -> torch.Tensor:
    """loss = score_neg - score_pos for a [2B,1,I,J,K,L] volume whose first B
    entries are the positive pairs and last B the negatives."""
    V = corr4d.shape[0]
    b = n_pos
    assert V == 2 * b
    i, j, k, l = corr4d.shape[2:]
    R, Cc = i * j, k * l
    if _ext.use_hip(corr4d) and normalization == "softmax":
        x3 = corr4d.reshape(V, R, Cc)
        wr, wc = _loss_weights(b, R, Cc, corr4d.device)
        return SoftmaxMaxScoreFn.apply(x3, wr, wc)
    pos = ref.match_score(corr4d[:b], normalization)
    neg = ref.match_score(corr4d[b:], normalization)
    return neg - pos


def match_score(corr4d: torch.Tensor, normalization: str | None = "softmax") -> torch.Tensor:
    """mean(scores_A + scores_B) / 2 of one batch (train.py:125-134)."""
    V = corr4d.shape[0]
    i, j, k, l = corr4d.shape[2:]
    R, Cc = i * j, k * l
    if _ext.use_hip(corr4d) and normalization == "softmax":
        wr = torch.full((V,), 1.0 / (2.0 * V * R), device=corr4d.device)
        wc = torch.full((V,), 1.0 / (2.0 * V * Cc), device=corr4d.device)
        return SoftmaxMaxScoreFn.apply(corr4d.reshape(V, R, Cc), wr, wc)
    return ref.match_score(corr4d, normalization)
