"""Image display helpers (reference lib/plot.py:6-29).

``plot_image`` undoes the ImageNet normalisation of a [3,H,W] (or batched)
tensor and shows it (or returns the uint8 HWC array); ``save_plot`` writes the
current figure without axes or margins.  matplotlib is imported lazily and the
Agg backend is used when no display is available.
"""
from __future__ import annotations

import numpy as np
import torch

from ..data.transforms import IMAGENET_MEAN, IMAGENET_STD


def _plt():
    import matplotlib

    if not matplotlib.get_backend() or "DISPLAY" not in __import__("os").environ:
        matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    return plt


def denormalize_image(im: torch.Tensor, batch_idx: int = 0) -> np.ndarray:
    """Normalised [3,H,W] / [B,3,H,W] tensor -> uint8 [H,W,3]."""
    if im.dim() == 4:
        im = im[batch_idx]
    mean = torch.tensor(IMAGENET_MEAN, dtype=torch.float32, device=im.device).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=torch.float32, device=im.device).view(3, 1, 1)
    x = (im.detach().float() * std + mean) * 255.0
    return x.clamp(0, 255).permute(1, 2, 0).cpu().numpy().astype(np.uint8)


def plot_image(im: torch.Tensor, batch_idx: int = 0, return_im: bool = False):
    arr = denormalize_image(im, batch_idx)
    if return_im:
        return arr
    plt = _plt()
    plt.imshow(arr)
    plt.show()
    return None


def save_plot(filename: str):
    plt = _plt()
    ax = plt.gca()
    ax.set_axis_off()
    plt.subplots_adjust(top=1, bottom=0, right=1, left=0, hspace=0, wspace=0)
    plt.margins(0, 0)
    ax.xaxis.set_major_locator(plt.NullLocator())
    ax.yaxis.set_major_locator(plt.NullLocator())
    plt.savefig(filename, bbox_inches="tight", pad_inches=0)
