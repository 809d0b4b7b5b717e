"""Image transforms (lib/normalization.py, lib/transformation.py).

The reference resizes with an identity ``affine_grid`` + ``grid_sample`` under
torch-0.3 semantics, i.e. bilinear sampling with ``align_corners=True``; that
is exactly ``F.interpolate(mode='bilinear', align_corners=True)``, which is what
``resize_bilinear`` uses.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def resize_bilinear(img: torch.Tensor, out_h: int, out_w: int) -> torch.Tensor:
    """[B,C,H,W] or [C,H,W] float -> resized, align_corners=True."""
    squeeze = img.dim() == 3
    x = img.unsqueeze(0) if squeeze else img
    y = F.interpolate(x.float(), size=(out_h, out_w), mode="bilinear", align_corners=True)
    return y.squeeze(0) if squeeze else y


class AffineTnf:
    """Affine warp with a [B,2,3] theta (identity by default), align_corners=True
    (lib/transformation.py:15-49)."""

    def __init__(self, out_h: int = 240, out_w: int = 240, use_cuda: bool = False):
        self.out_h, self.out_w = out_h, out_w
        self.theta_identity = torch.tensor([[[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]]])

    def __call__(self, image_batch, theta_batch=None, out_h=None, out_w=None):
        b = 1 if image_batch is None else image_batch.shape[0]
        oh, ow = out_h or self.out_h, out_w or self.out_w
        if theta_batch is None:
            theta_batch = self.theta_identity.to(image_batch.device).expand(b, 2, 3)
        grid = F.affine_grid(theta_batch.float(), [b, 3, oh, ow], align_corners=True)
        return F.grid_sample(image_batch.float(), grid, mode="bilinear", align_corners=True)


def normalize_image(image: torch.Tensor, forward: bool = True, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """(x - mean) / std or its inverse, for [C,H,W] or [B,C,H,W] (lib/normalization.py:29-50)."""
    shape = (1, 3, 1, 1) if image.dim() == 4 else (3, 1, 1)
    m = torch.tensor(mean, dtype=image.dtype, device=image.device).view(shape)
    s = torch.tensor(std, dtype=image.dtype, device=image.device).view(shape)
    return (image - m) / s if forward else image * s + m


class NormalizeImageDict:
    """/255 (optional) then ImageNet normalisation of the given keys (lib/normalization.py:5-26)."""

    def __init__(self, image_keys, normalizeRange: bool = True):  # noqa: N803
        self.image_keys = image_keys
        self.normalizeRange = normalizeRange

    def __call__(self, sample):
        for key in self.image_keys:
            x = sample[key].float()
            if self.normalizeRange:
                x = x / 255.0
            sample[key] = normalize_image(x)
        return sample


def read_image(path: str) -> np.ndarray:
    """HxWx3 uint8 (grayscale expanded to 3 channels; skimage is not required)."""
    from PIL import Image

    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB") if im.mode not in ("RGB", "L") else im)
    if arr.ndim == 2:
        arr = np.repeat(arr[:, :, None], 3, axis=2)
    return arr


def to_chw_float(arr: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1))).float()


def gpu_normalize_resize(imgs_uint8: torch.Tensor, out_h: int, out_w: int) -> torch.Tensor:
    """Batched uint8 [B,3,H,W] -> normalised float [B,3,out_h,out_w] on the
    current device (the GPU-side alternative to per-sample CPU resizing)."""
    x = imgs_uint8.float() / 255.0
    x = resize_bilinear(x, out_h, out_w)
    return normalize_image(x)
