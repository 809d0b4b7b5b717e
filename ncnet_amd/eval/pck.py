"""PCK keypoint-transfer metric (lib/eval_util.py), vectorised over the batch."""
from __future__ import annotations

import numpy as np
import torch

from .point_tnf import PointsToPixelCoords, PointsToUnitCoords, bilinearInterpPointTnf


def pck(source_points: torch.Tensor, warped_points: torch.Tensor, L_pck: torch.Tensor, alpha: float = 0.1):  # noqa: N803
    """Fraction of valid points with ||p - p_hat|| <= alpha * L_pck, per sample
    (lib/eval_util.py:12-24).  Points are [b, 2, N] padded with -1."""
    valid = (source_points[:, 0, :] != -1) & (source_points[:, 1, :] != -1)
    d = torch.sqrt(((source_points - warped_points) ** 2).sum(1))
    correct = (d <= L_pck.view(-1, 1) * alpha) & valid
    n = valid.sum(1).clamp(min=1)
    out = correct.sum(1).float() / n.float()
    out[valid.sum(1) == 0] = float("nan")
    return out


def pck_metric(batch, batch_start_idx, matches, stats, args=None, use_cuda=True, alpha: float = 0.1):
    """Transfer target keypoints to the source through ``matches`` and record
    PCK in ``stats['point_tnf']['pck']`` (lib/eval_util.py:27-51)."""
    source_im_size, target_im_size = batch["source_im_size"], batch["target_im_size"]
    source_points, target_points = batch["source_points"], batch["target_points"]
    target_points_norm = PointsToUnitCoords(target_points, target_im_size)
    warped_norm = bilinearInterpPointTnf(matches, target_points_norm)
    warped = PointsToPixelCoords(warped_norm, source_im_size)
    res = pck(source_points, warped, batch["L_pck"].view(-1).to(warped.dtype), alpha)
    b = res.shape[0]
    stats["point_tnf"]["pck"][batch_start_idx:batch_start_idx + b] = res.detach().cpu().numpy().reshape(-1, 1)
    return stats


def summarize(stats) -> dict:
    r = stats["point_tnf"]["pck"]
    good = np.flatnonzero((r != -1) * ~np.isnan(r))
    return {"total": int(r.size), "valid": int(good.size), "pck": float(np.mean(r[good])) if good.size else float("nan")}
