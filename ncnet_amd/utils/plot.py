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


def _gray(img: np.ndarray) -> np.ndarray:
    img = np.asarray(img, np.float64)
    if img.ndim == 3:
        img = img[..., 0] * 0.2989 + img[..., 1] * 0.5870 + img[..., 2] * 0.1140
    return img


def _resize_gray(img: np.ndarray, scale: float) -> np.ndarray:
    if scale == 1.0:
        return img
    t = torch.as_tensor(img, dtype=torch.float32)[None, None]
    h, w = max(1, int(round(img.shape[0] * scale))), max(1, int(round(img.shape[1] * scale)))
    return torch.nn.functional.interpolate(t, size=(h, w), mode="bilinear", align_corners=False)[0, 0].numpy()


def side_by_side(I1: np.ndarray, I2: np.ndarray, gap: int = 0):
    """Grey images scaled to the smaller height and concatenated horizontally
    (the layout of show_matches2_horizontal.m:12-25 / parfor_nc4d_PV.m:76-92).
    Returns (canvas, scale1, scale2, x-offset of the second image)."""
    g1, g2 = _gray(I1), _gray(I2)
    if g1.shape[0] <= g2.shape[0]:
        s1, s2 = 1.0, g1.shape[0] / g2.shape[0]
    else:
        s1, s2 = g2.shape[0] / g1.shape[0], 1.0
    g1, g2 = _resize_gray(g1, s1), _resize_gray(g2, s2)
    h = min(g1.shape[0], g2.shape[0])
    canvas = np.concatenate([g1[:h], np.full((h, gap), np.nan), g2[:h]], 1)
    return canvas, s1, s2, g1.shape[1] + gap


def show_matches_horizontal(I1, I2, x1, y1, x2, y2, inliers=None, out: str | None = None,
                            color="y", linewidth=0.5):
    """Match visualisation (lib_matlab/show_matches2_horizontal.m): both images
    side by side (grey), all matches as blue dots, inliers as green dots joined
    by lines.  Coordinates are pixels of the original images.  Saves to
    ``out`` when given; returns the figure."""
    plt = _plt()
    canvas, s1, s2, xo = side_by_side(I1, I2, gap=10)
    fig = plt.figure(figsize=(canvas.shape[1] / 100.0, canvas.shape[0] / 100.0), dpi=100)
    ax = fig.add_axes([0, 0, 1, 1])
    ax.imshow(canvas, cmap="gray")
    ax.set_axis_off()
    x1, y1, x2, y2 = (np.asarray(a, np.float64) for a in (x1, y1, x2, y2))
    ax.scatter(np.r_[s1 * x1, s2 * x2 + xo], np.r_[s1 * y1, s2 * y2], s=10, c="b")
    if inliers is not None:
        m = np.asarray(inliers, bool)
        ax.scatter(np.r_[s1 * x1[m], s2 * x2[m] + xo], np.r_[s1 * y1[m], s2 * y2[m]], s=10, c="g")
        for a, b, c, d in zip(s1 * x1[m], s1 * y1[m], s2 * x2[m] + xo, s2 * y2[m]):
            ax.plot([a, c], [b, d], color=color, linewidth=linewidth)
    if out:
        fig.savefig(out)
    return fig


def plot_localization_curves(methods, out: str, thresholds=None, title="InLoc (DUC1 + DUC2)"):
    """Localization-rate curves (lib_matlab/generate_ncnet_plot.m +
    ht_plotcurve_WUSTL.m:84-112): ``methods`` is a list of dicts with keys
    ``rate`` (fraction per threshold), ``description`` and optional ``marker``
    (e.g. 'DensePE + NCNet' '--b', 'InLoc + NCNet' '--c').  Saves ``out``."""
    from ..eval.localization import DEFAULT_THRESHOLDS

    thr = np.asarray(DEFAULT_THRESHOLDS if thresholds is None else thresholds)
    plt = _plt()
    fig, ax = plt.subplots(figsize=(6, 4.5))
    for m in methods:
        ax.plot(thr, 100.0 * np.asarray(m["rate"]), m.get("marker", "-"), label=m["description"], linewidth=2)
    ax.set_xlabel("Distance threshold [meters]")
    ax.set_ylabel("Correctly localized queries [%]")
    ax.set_xlim(thr[0], thr[-1])
    ax.set_ylim(0, 80)
    ax.grid(True)
    ax.legend(loc="lower right")
    ax.set_title(title)
    fig.savefig(out, bbox_inches="tight")
    return fig
