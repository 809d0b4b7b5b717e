"""Match extraction and point transfer (lib/point_tnf.py).

``corr_to_matches`` returns, for every cell of one image, the best match in
the other, optionally after a softmax over the candidates, with relocalization
offsets decoded to full resolution.  On GPU the per-row / per-column
max, first-argmax and softmax denominators come from the HIP online-softmax
statistics kernels in one pass each; the grid lookups are tiny gathers.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import _ext


def normalize_axis(x, L):
    return (x - 1 - (L - 1) / 2) * 2 / (L - 1)


def unnormalize_axis(x, L):
    return x * (L - 1) / 2 + 1 + (L - 1) / 2


def _best(mat: torch.Tensor, dim: int, do_softmax: bool):
    """mat [b, R, C] -> (score, index) of the best entry along ``dim``."""
    if _ext.use_hip(mat) and mat.dtype == torch.float32:
        x = mat.contiguous()
        b, R, C = x.shape
        n = C if dim == 1 else R
        mx = torch.empty((b, n), dtype=torch.float32, device=x.device)
        arg = torch.empty((b, n), dtype=torch.int32, device=x.device)
        se = torch.empty((b, n), dtype=torch.float32, device=x.device) if do_softmax else None
        if dim == 1:
            _ext.ext().stats_cols(x, mx, arg, se, 1)
        else:
            _ext.ext().stats_rows(x, mx, arg, se, 1)
        score = (1.0 / se) if do_softmax else mx
        return score, arg.long()
    v = torch.softmax(mat, dim=dim) if do_softmax else mat
    score, idx = torch.max(v, dim=dim)
    return score, idx


def best_both(corr4d, do_softmax: bool):
    """The (score, index) of the best entry along both directions of the
    volume in one pass (stats2d) -> ((score_B, idx_B), (score_A, idx_A)), or
    None where stats2d does not apply (CPU, or rows not a 16-byte multiple)."""
    b, _, fs1, fs2, fs3, fs4 = corr4d.shape
    mat = corr4d.reshape(b, fs1 * fs2, fs3 * fs4)
    if not (_ext.use_hip(mat) and mat.dtype == torch.float32):
        return None
    x = mat.contiguous()
    R, C = x.shape[1], x.shape[2]
    f = dict(dtype=torch.float32, device=x.device)
    rmx, cmx = torch.empty((b, R), **f), torch.empty((b, C), **f)
    rarg = torch.empty((b, R), dtype=torch.int32, device=x.device)
    carg = torch.empty((b, C), dtype=torch.int32, device=x.device)
    rse = torch.empty((b, R), **f) if do_softmax else None
    cse = torch.empty((b, C), **f) if do_softmax else None
    if not _ext.ext().stats2d(x, rmx, rarg, rse, cmx, carg, cse, 1 if do_softmax else 0):
        return None
    col = ((1.0 / cse) if do_softmax else cmx, carg.long())
    row = ((1.0 / rse) if do_softmax else rmx, rarg.long())
    return col, row


def corr_to_matches(corr4d, delta4d=None, k_size=1, do_softmax=False, scale="centered", return_indices=False,
                    invert_matching_direction=False, best=None):
    """Matches from a [b,1,fs1,fs2,fs3,fs4] volume (lib/point_tnf.py:12-80).

    B->A (default): for each B cell the best A cell; A->B with
    ``invert_matching_direction``.  Coordinates on a linspace grid in
    [-1,1] ('centered') or [0,1] ('positive') at resolution fs*k_size."""
    b, ch, fs1, fs2, fs3, fs4 = corr4d.shape
    dev = corr4d.device
    lo = -1.0 if scale == "centered" else 0.0
    ya = torch.linspace(lo, 1, fs1 * k_size, device=dev)
    xa = torch.linspace(lo, 1, fs2 * k_size, device=dev)
    yb = torch.linspace(lo, 1, fs3 * k_size, device=dev)
    xb = torch.linspace(lo, 1, fs4 * k_size, device=dev)
    mat = corr4d.reshape(b, fs1 * fs2, fs3 * fs4)
    if mat.dtype != torch.float32:
        mat = mat.float()
    if invert_matching_direction:
        score, idx = best if best is not None else _best(mat, 2, do_softmax)   # per A cell, best B
        ia = torch.arange(fs1 * fs2, device=dev).expand(b, -1)
        iA, jA = ia // fs2, ia % fs2
        iB, jB = idx // fs4, idx % fs4
    else:
        score, idx = best if best is not None else _best(mat, 1, do_softmax)   # per B cell, best A
        ib = torch.arange(fs3 * fs4, device=dev).expand(b, -1)
        iB, jB = ib // fs4, ib % fs4
        iA, jA = idx // fs2, idx % fs2
    if delta4d is not None:
        bi = torch.arange(b, device=dev).view(b, 1).expand_as(iA)
        if torch.is_tensor(delta4d):
            # packed 2-bit offsets (ops/correlation.py decode_offsets layout), decoded
            # only at the matched cells instead of over the whole volume
            code = delta4d.reshape(b, fs1, fs2, fs3, fs4)[bi, iA, jA, iB, jB].long()
            ddi, ddj, ddk, ddl = (code >> 6) & 3, (code >> 4) & 3, (code >> 2) & 3, code & 3
        else:
            di, dj, dk, dl = (d.reshape(b, fs1, fs2, fs3, fs4) for d in delta4d)
            ddi = di[bi, iA, jA, iB, jB]
            ddj = dj[bi, iA, jA, iB, jB]
            ddk = dk[bi, iA, jA, iB, jB]
            ddl = dl[bi, iA, jA, iB, jB]
        iA, jA = iA * k_size + ddi, jA * k_size + ddj
        iB, jB = iB * k_size + ddk, jB * k_size + ddl
    xA, yA = xa[jA], ya[iA]
    xB, yB = xb[jB], yb[iB]
    if return_indices:
        return xA, yA, xB, yB, score, iA, jA, iB, jB
    return xA, yA, xB, yB, score


def nearestNeighPointTnf(matches, target_points_norm):  # noqa: N802
    """Nearest-neighbour point transfer (lib/point_tnf.py:82-94)."""
    xA, yA, xB, yB = matches
    dx = target_points_norm[:, 0, :].unsqueeze(1) - xB.unsqueeze(2)
    dy = target_points_norm[:, 1, :].unsqueeze(1) - yB.unsqueeze(2)
    idx = torch.sqrt(dx * dx + dy * dy).min(dim=1)[1]
    wx = torch.gather(xA, 1, idx)
    wy = torch.gather(yA, 1, idx)
    return torch.stack((wx, wy), dim=1)


def bilinearInterpPointTnf(matches, target_points_norm):  # noqa: N802
    """Bilinear keypoint transfer over the (square) B grid (lib/point_tnf.py:96-148)."""
    xA, yA, xB, yB = matches
    fs = int(round(np.sqrt(xB.shape[-1])))
    b, _, n = target_points_norm.shape
    grid = torch.linspace(-1, 1, fs, device=xB.device).view(1, fs, 1)
    xm = ((target_points_norm[:, 0, :].unsqueeze(1) - grid) > 0).long().sum(1, keepdim=True) - 1
    xm = xm.clamp(min=0)
    ym = ((target_points_norm[:, 1, :].unsqueeze(1) - grid) > 0).long().sum(1, keepdim=True) - 1
    ym = ym.clamp(min=0)
    xp, yp = xm + 1, ym + 1
    # the reference indexes beyond the grid for points on the last cell edge; clamp like fs-1
    xp, yp = xp.clamp(max=fs - 1), yp.clamp(max=fs - 1)
    toidx = lambda x, y: y * fs + x  # noqa: E731
    idx_mm, idx_pp, idx_pm, idx_mp = toidx(xm, ym), toidx(xp, yp), toidx(xp, ym), toidx(xm, yp)
    XB, YB = xB.reshape(b, -1), yB.reshape(b, -1)
    XA, YA = xA.reshape(b, -1), yA.reshape(b, -1)

    def topoint(idx, X, Y):
        i = idx.view(b, n)
        return torch.stack((torch.gather(X, 1, i), torch.gather(Y, 1, i)), dim=1)

    P_mm, P_pp, P_pm, P_mp = (topoint(i, XB, YB) for i in (idx_mm, idx_pp, idx_pm, idx_mp))
    mult = lambda x: x[:, 0, :] * x[:, 1, :]  # noqa: E731
    f_pp = mult(torch.abs(target_points_norm - P_mm))
    f_mm = mult(torch.abs(target_points_norm - P_pp))
    f_mp = mult(torch.abs(target_points_norm - P_pm))
    f_pm = mult(torch.abs(target_points_norm - P_mp))
    Q_mm, Q_pp, Q_pm, Q_mp = (topoint(i, XA, YA) for i in (idx_mm, idx_pp, idx_pm, idx_mp))
    num = Q_mm * f_mm.unsqueeze(1) + Q_pp * f_pp.unsqueeze(1) + Q_mp * f_mp.unsqueeze(1) + Q_pm * f_pm.unsqueeze(1)
    den = (f_pp + f_mm + f_mp + f_pm).unsqueeze(1)
    return num / den


def PointsToUnitCoords(P, im_size):  # noqa: N802
    h, w = im_size[:, 0], im_size[:, 1]
    out = P.clone()
    out[:, 0, :] = normalize_axis(P[:, 0, :], w.unsqueeze(1).expand_as(P[:, 0, :]))
    out[:, 1, :] = normalize_axis(P[:, 1, :], h.unsqueeze(1).expand_as(P[:, 1, :]))
    return out


def PointsToPixelCoords(P, im_size):  # noqa: N802
    h, w = im_size[:, 0], im_size[:, 1]
    out = P.clone()
    out[:, 0, :] = unnormalize_axis(P[:, 0, :], w.unsqueeze(1).expand_as(P[:, 0, :]))
    out[:, 1, :] = unnormalize_axis(P[:, 1, :], h.unsqueeze(1).expand_as(P[:, 1, :]))
    return out
