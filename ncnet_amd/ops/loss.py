"""Weak-supervision score (train.py:110-156) with a fused HIP forward/backward.

All three normalisations of the reference (train.py:111-116) run on the same
single-pass HIP statistics (max, first argmax, and a sum) plus one
closed-form backward kernel:

* ``'softmax'`` (default): ``max_j softmax(x)_j = 1 / sum_j exp(x_j - max x)``,
  ``ds/dx_j = s (delta_{j, argmax} - softmax_j)``;
* ``'l1'``: ``max_j x_j / (sum x + eps) = max x / (sum x + eps)`` (eps 1e-4;
  the volumes are non-negative -- ReLU'd NC outputs after MutualMatching -- so
  the positive denominator keeps the argmax), ``ds/dx_j = delta_{j, argmax} / D - max / D^2``;
* ``None``: ``max x``, ``ds/dx_j = delta_{j, argmax}``.
"""
from __future__ import annotations

import torch

from .. import config as _config
from . import _ext
from . import reference as ref


_NORM = {"softmax": 1, "l1": 2, None: 0}


def _row_col_stats(x3: torch.Tensor, norm: int):
    C = _ext.ext()
    V, R, Cc = x3.shape
    f = dict(dtype=torch.float32, device=x3.device)
    rmax, rse = torch.empty((V, R), **f), torch.empty((V, R), **f)
    cmax, cse = torch.empty((V, Cc), **f), torch.empty((V, Cc), **f)
    rarg = torch.empty((V, R), dtype=torch.int32, device=x3.device)
    carg = torch.empty((V, Cc), dtype=torch.int32, device=x3.device)
    sum_kind = {1: 1, 2: 2, 0: 0}[norm]
    # one pass for both directions when rows are 16-byte multiples (stats2d)
    if not (_config.RUNTIME.stats2d and C.stats2d(x3, rmax, rarg, rse, cmax, carg, cse, sum_kind)):
        C.stats_rows(x3, rmax, rarg, rse if sum_kind else None, sum_kind)
        C.stats_cols(x3, cmax, carg, cse if sum_kind else None, sum_kind)
    if not sum_kind:
        rse.zero_()
        cse.zero_()
    return rmax, rarg, rse, cmax, carg, cse


class SoftmaxMaxScoreFn(torch.autograd.Function):
    """sum_v wr[v] * sum_rows s_row + wc[v] * sum_cols s_col, s = the max of the
    normalised row / column (norm 1 softmax, 2 l1, 0 None)."""

    @staticmethod
    def forward(ctx, x3, wr, wc, norm=1):
        x3 = x3.float().contiguous()
        st = _row_col_stats(x3, norm)
        rmax, rarg, rse, cmax, carg, cse = st
        # one launch for the weighted score sum (was 7 small PyTorch kernels on the step's critical path)
        val = torch.empty((), dtype=torch.float32, device=x3.device)
        _ext.ext().score_sum(rmax, rse, cmax, cse, wr.float().contiguous(), wc.float().contiguous(), val, norm,
                             ref.L1_EPS)
        ctx.norm = norm
        ctx.save_for_backward(x3, wr, wc, *st)
        return val

    @staticmethod
    def backward(ctx, g):
        x3, wr, wc, rmax, rarg, rse, cmax, carg, cse = ctx.saved_tensors
        gx = torch.empty_like(x3)
        # the incoming gradient scales inside the kernel (no extra pass over the volume)
        _ext.ext().softmax_max_bwd(x3, rmax, rarg, rse, cmax, carg, cse, wr.float().contiguous(),
                                   wc.float().contiguous(), gx, ctx.norm, ref.L1_EPS, g.float().contiguous().reshape(1))
        return gx, None, None, None


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
    if normalization not in _NORM:
        raise ValueError(f"normalization must be 'softmax', 'l1' or None, got {normalization!r}")
    if _ext.use_hip(corr4d):
        x3 = corr4d.reshape(V, R, Cc)
        wr, wc = _loss_weights(b, R, Cc, corr4d.device)
        return SoftmaxMaxScoreFn.apply(x3, wr, wc, _NORM[normalization])
    pos = ref.match_score(corr4d[:b], normalization)
    neg = ref.match_score(corr4d[b:], normalization)
    return neg - pos


def match_score(corr4d: torch.Tensor, normalization: str | None = "softmax") -> torch.Tensor:
    """mean(scores_A + scores_B) / 2 of one batch (train.py:125-134)."""
    V = corr4d.shape[0]
    i, j, k, l = corr4d.shape[2:]
    R, Cc = i * j, k * l
    if normalization not in _NORM:
        raise ValueError(f"normalization must be 'softmax', 'l1' or None, got {normalization!r}")
    if _ext.use_hip(corr4d):
        wr = torch.full((V,), 1.0 / (2.0 * V * R), device=corr4d.device)
        wc = torch.full((V,), 1.0 / (2.0 * V * Cc), device=corr4d.device)
        return SoftmaxMaxScoreFn.apply(corr4d.reshape(V, R, Cc), wr, wc, _NORM[normalization])
    return ref.match_score(corr4d, normalization)
