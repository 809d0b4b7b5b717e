"""Pure-PyTorch oracles for every NC-Net tensor primitive.

These run on any device (the CPU path of the framework and the numerics
reference for every HIP kernel test).  They re-specify the reference's
behaviour explicitly, including the places where the reference silently
depends on torch-0.3 semantics:

* ``feature_l2norm``      -- lib/model.py:14-17 (eps 1e-6 *inside* the sqrt)
* ``correlation_4d``      -- lib/model.py:106-115 ('4D' FeatureCorrelation)
* ``correlation_3d``      -- lib/model.py:97-105 ('3D' legacy mode)
* ``mutual_matching``     -- lib/model.py:155-175
* ``maxpool4d``           -- lib/model.py:177-191, but batch-correct and with
                             integer offsets (the reference folds the batch into
                             the max and returns float offsets on modern torch)
* ``conv4d``              -- lib/conv4d.py:11-51 semantics ("same" zero padding,
                             stride 1, bias added once), computed as k batched
                             conv3d calls instead of an h*k Python loop
* ``conv4d_sliced``       -- the reference *algorithm* (h*k conv3d launches,
                             lib/conv4d.py:39-48), kept only as the measured
                             baseline for bench.py
* ``softmax_max_scores``  -- the weak-loss scores of train.py:121-134

Weight layout: Conv4d weights are stored the way the reference checkpoints
store them, pre-permuted to ``[k, out, in, k, k, k]`` (lib/conv4d.py:75-77).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

L2NORM_EPS = 1e-6
MUTUAL_EPS = 1e-5
L1_EPS = 1e-4


def feature_l2norm(feature: torch.Tensor, dim: int = 1) -> torch.Tensor:
    """f / sqrt(sum_c f^2 + 1e-6)  (lib/model.py:14-17)."""
    norm = torch.sqrt(torch.sum(feature * feature, dim=dim, keepdim=True) + L2NORM_EPS)
    return feature / norm


def correlation_4d(feature_a: torch.Tensor, feature_b: torch.Tensor) -> torch.Tensor:
    """[b,c,hA,wA] x [b,c,hB,wB] -> [b,1,hA,wA,hB,wB] (lib/model.py:106-115)."""
    b, c, ha, wa = feature_a.shape
    _, _, hb, wb = feature_b.shape
    fa = feature_a.reshape(b, c, ha * wa).transpose(1, 2)
    fb = feature_b.reshape(b, c, hb * wb)
    return torch.bmm(fa, fb).view(b, 1, ha, wa, hb, wb)


def correlation_3d(feature_a: torch.Tensor, feature_b: torch.Tensor) -> torch.Tensor:
    """Legacy CNNGeometric layout [b, h*w, h, w] indexed
    [batch, idx_A = row_A + h*col_A, row_B, col_B] (lib/model.py:97-105)."""
    b, c, h, w = feature_a.shape
    fa = feature_a.transpose(2, 3).reshape(b, c, h * w)
    fb = feature_b.reshape(b, c, h * w).transpose(1, 2)
    mul = torch.bmm(fb, fa)  # [b, hB*wB, idx_A]
    return mul.view(b, h, w, h * w).permute(0, 3, 1, 2)


def mutual_matching(corr4d: torch.Tensor) -> torch.Tensor:
    """Soft mutual nearest-neighbour filter (lib/model.py:155-175).

    out = c * ((c / (max_A c + eps)) * (c / (max_B c + eps))); the product of
    the two ratios is taken first, exactly as the reference parenthesises it,
    which keeps the output exactly symmetric under the A<->B swap.
    """
    b, ch, i, j, k, l = corr4d.shape
    c_b = corr4d.reshape(b, i * j, k, l)        # max over A positions per B cell
    c_a = corr4d.reshape(b, i, j, k * l)        # max over B positions per A cell
    max_b = c_b.max(dim=1, keepdim=True)[0]
    max_a = c_a.max(dim=3, keepdim=True)[0]
    ratio_b = (c_b / (max_b + MUTUAL_EPS)).reshape(b, 1, i, j, k, l)
    ratio_a = (c_a / (max_a + MUTUAL_EPS)).reshape(b, 1, i, j, k, l)
    return corr4d * (ratio_a * ratio_b)


def maxpool4d(corr4d: torch.Tensor, k_size: int):
    """4D max pooling with stride = kernel = k, batch-correct, integer offsets.

    Returns ``(pooled [b,1,I/k,J/k,K/k,L/k], (di, dj, dk, dl))`` where each
    offset tensor has the pooled shape and holds the in-window argmax position
    (lib/model.py:177-191).  Ties resolve to the first index in (i,j,k,l)
    lexicographic order, the order in which the reference enumerates slices.
    """
    b, ch, i, j, k, l = corr4d.shape
    assert ch == 1
    s = k_size
    x = corr4d.reshape(b, i // s, s, j // s, s, k // s, s, l // s, s)
    x = x.permute(0, 1, 3, 5, 7, 2, 4, 6, 8).reshape(b, i // s, j // s, k // s, l // s, s ** 4)
    vals, idx = x.max(dim=-1)
    d_l = idx % s
    d_k = (idx // s) % s
    d_j = (idx // (s * s)) % s
    d_i = idx // (s * s * s)
    vals = vals.unsqueeze(1)
    return vals, tuple(t.unsqueeze(1) for t in (d_i, d_j, d_k, d_l))


def conv4d_weight_to_std(weight_ref: torch.Tensor) -> torch.Tensor:
    """[k, out, in, k, k, k] (checkpoint layout) -> [out, in, k, k, k, k]."""
    return weight_ref.permute(1, 2, 0, 3, 4, 5)


def conv4d_weight_from_std(weight_std: torch.Tensor) -> torch.Tensor:
    """[out, in, k, k, k, k] -> [k, out, in, k, k, k] (checkpoint layout)."""
    return weight_std.permute(2, 0, 1, 3, 4, 5).contiguous()


def conv4d(x: torch.Tensor, weight_ref: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """"Same"-padded stride-1 4D cross-correlation.

    x: [N, Cin, I, J, K, L]; weight_ref: [k, Cout, Cin, k, k, k]; bias: [Cout].
    Computed as k conv3d calls, each over the whole (N*I) batch of 3D slices,
    summing the first-axis taps by shifting a once-padded view (the reference
    instead loops in Python over every output slice: lib/conv4d.py:39-48).
    """
    n, cin, i, j, k, l = x.shape
    ks = weight_ref.shape[0]
    cout = weight_ref.shape[1]
    p = ks // 2
    xp = F.pad(x, (0, 0, 0, 0, 0, 0, p, p))  # pad the I axis only
    out = None
    for di in range(ks):
        xs = xp[:, :, di:di + i].permute(0, 2, 1, 3, 4, 5).reshape(n * i, cin, j, k, l)
        o = F.conv3d(xs, weight_ref[di], bias=None, padding=p)
        out = o if out is None else out + o
    out = out.reshape(n, i, cout, j, k, l).permute(0, 2, 1, 3, 4, 5)
    if bias is not None:
        out = out + bias.view(1, cout, 1, 1, 1, 1)
    return out.contiguous()


def conv4d_sliced(x: torch.Tensor, weight_ref: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """The reference *algorithm* (lib/conv4d.py:39-48): one conv3d per output
    slice and per first-axis tap, i.e. I*k launches.  Used only as the
    measured "reference-algorithm" baseline in bench.py."""
    n, cin, i, j, k, l = x.shape
    ks = weight_ref.shape[0]
    p = ks // 2
    data = x.permute(2, 0, 1, 3, 4, 5).contiguous()          # [I, N, Cin, J, K, L]
    zeros = data.new_zeros((p,) + tuple(data.shape[1:]))
    padded = torch.cat((zeros, data, zeros), 0)
    slices = []
    for ii in range(i):
        acc = F.conv3d(padded[ii + p], weight_ref[p], bias=bias, padding=p)
        for t in range(1, p + 1):
            acc = acc + F.conv3d(padded[ii + p - t], weight_ref[p - t], padding=p)
            acc = acc + F.conv3d(padded[ii + p + t], weight_ref[p + t], padding=p)
        slices.append(acc)
    return torch.stack(slices, 0).permute(1, 2, 0, 3, 4, 5).contiguous()


def swap_ab(x: torch.Tensor) -> torch.Tensor:
    """[N, C, I, J, K, L] -> [N, C, K, L, I, J] (A<->B swap, lib/model.py:147)."""
    return x.permute(0, 1, 4, 5, 2, 3)


def neigh_consensus(x: torch.Tensor, weights, biases, symmetric: bool = True, conv=conv4d) -> torch.Tensor:
    """Stack of Conv4d+ReLU, optionally symmetric (lib/model.py:143-153)."""
    def stack(v):
        for w, b in zip(weights, biases):
            v = F.relu(conv(v, w, b))
        return v
    if symmetric:
        return stack(x) + swap_ab(stack(swap_ab(x)))
    return stack(x)


def softmax_max_scores(corr4d: torch.Tensor, normalization: str | None = "softmax"):
    """Per-cell matching scores of train.py:121-134.

    Returns (scores_A, scores_B): scores_B[b, kB] = max over A positions of the
    normalised column, scores_A[b, kA] = max over B positions of the row.
    """
    b = corr4d.shape[0]
    i, j, k, l = corr4d.shape[2:]
    mat = corr4d.reshape(b, i * j, k * l)

    def norm(v, dim):
        if normalization is None:
            return v
        if normalization == "softmax":
            return torch.softmax(v, dim=dim)
        if normalization == "l1":
            return v / (v.sum(dim=dim, keepdim=True) + L1_EPS)
        raise ValueError(normalization)

    scores_b = norm(mat, 1).max(dim=1)[0]  # per B cell, over A
    scores_a = norm(mat, 2).max(dim=2)[0]  # per A cell, over B
    return scores_a, scores_b


def match_score(corr4d: torch.Tensor, normalization: str | None = "softmax") -> torch.Tensor:
    """mean(scores_A + scores_B) / 2 (train.py:134); needs square maps like the
    reference (train.py:124) only when the two score vectors differ in length,
    in which case each direction is averaged separately."""
    sa, sb = softmax_max_scores(corr4d, normalization)
    if sa.shape == sb.shape:
        return torch.mean(sa + sb) / 2
    return (sa.mean() + sb.mean()) / 2
