"""Pair datasets (lib/im_pair_dataset.py, lib/pf_dataset.py) and synthetic pairs.

CSV formats:
* train / val: ``source_image,target_image,class,flip``
* PF-Pascal test: ``source_image,target_image,class,XA,YA,XB,YB`` with ``;``
  separated point lists.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import torch
from torch.utils.data import Dataset

from .transforms import read_image, resize_bilinear, to_chw_float

PF_CATEGORIES = ["aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair", "cow",
                 "diningtable", "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa", "train",
                 "tvmonitor"]


class ImagePairDataset(Dataset):
    """Weakly supervised image pairs (lib/im_pair_dataset.py:11-93)."""

    def __init__(self, dataset_csv_path, dataset_csv_file, dataset_image_path, dataset_size=0,
                 output_size=(240, 240), transform=None, random_crop=False, gpu_resize=False):
        """``gpu_resize``: return the decoded (cropped / flipped) images as
        uint8 CHW tensors of their own size and let the consumer resize +
        normalise the batch on the GPU (``gpu_pair_batch``; collate with
        ``collate_uint8_pairs``) -- the DataLoader workers then only decode."""
        self.random_crop = random_crop
        self.gpu_resize = gpu_resize
        self.out_h, self.out_w = output_size
        data = pd.read_csv(os.path.join(dataset_csv_path, dataset_csv_file))
        if dataset_size:
            data = data.iloc[: min(dataset_size, len(data))]
        self.img_A_names = data.iloc[:, 0].tolist()
        self.img_B_names = data.iloc[:, 1].tolist()
        self.set = data.iloc[:, 2].to_numpy()
        self.flip = data.iloc[:, 3].to_numpy().astype("int")
        self.dataset_image_path = dataset_image_path
        self.transform = transform

    def __len__(self):
        return len(self.img_A_names)

    def get_image(self, name, flip):
        image = read_image(os.path.join(self.dataset_image_path, name))
        if self.random_crop:
            h, w, _ = image.shape
            top = np.random.randint(h // 4)
            bottom = int(3 * h / 4 + np.random.randint(h // 4))
            left = np.random.randint(w // 4)
            right = int(3 * w / 4 + np.random.randint(w // 4))
            image = image[top:bottom, left:right, :]
        if flip:
            image = np.flip(image, 1)
        im_size = torch.tensor(image.shape, dtype=torch.float32)
        if self.gpu_resize:          # HWC uint8 as decoded; packed per batch by collate_uint8_pairs
            return torch.from_numpy(np.ascontiguousarray(image)), im_size
        img = resize_bilinear(to_chw_float(image), self.out_h, self.out_w)
        return img, im_size

    def __getitem__(self, idx):
        a, sa = self.get_image(self.img_A_names[idx], self.flip[idx])
        b, sb = self.get_image(self.img_B_names[idx], self.flip[idx])
        sample = {"source_image": a, "target_image": b, "source_im_size": sa, "target_im_size": sb,
                  "set": int(self.set[idx])}
        if self.transform and not self.gpu_resize:
            sample = self.transform(sample)
        return sample


def collate_uint8_pairs(samples):
    """Batch of ``gpu_resize`` samples (runs in the DataLoader workers): the
    decoded HWC uint8 pixels of all 2B images are packed into ONE byte buffer
    ``pixels`` with a table ``pixel_meta`` [2B, 3] = (byte offset, H, W)
    (sources first, then targets) -- one pinned tensor, one host->device copy;
    everything else is stacked."""
    imgs = [s["source_image"] for s in samples] + [s["target_image"] for s in samples]
    sizes = [int(x.numel()) for x in imgs]
    offs = np.concatenate(([0], np.cumsum(sizes)[:-1])).astype(np.int64)
    meta = torch.tensor([[o, x.shape[0], x.shape[1]] for o, x in zip(offs, imgs)], dtype=torch.int64)
    out = {"pixels": torch.cat([x.reshape(-1) for x in imgs]), "pixel_meta": meta}
    for k in samples[0]:
        if k in ("source_image", "target_image"):
            continue
        vals = [s[k] for s in samples]
        out[k] = torch.stack(vals) if torch.is_tensor(vals[0]) else torch.tensor(vals)
    return out


def gpu_pair_batch(batch, device, out_h: int, out_w: int):
    """Move a ``collate_uint8_pairs`` batch to ``device`` (uint8 pixels: 4x
    fewer bytes than float, one non-blocking copy) and resize + normalise all
    images there in one HIP launch (csrc/dataprep.hip): bilinear with
    align_corners=True as the reference's identity AffineTnf
    (lib/transformation.py), then ImageNet normalisation
    (lib/normalization.py).  On CPU the same math runs through torch."""
    from .transforms import IMAGENET_MEAN, IMAGENET_STD, gpu_normalize_resize
    from ..ops import _ext
    pix, meta = batch["pixels"], batch["pixel_meta"]
    n = meta.shape[0]
    ends = meta[:, 0] + meta[:, 1] * meta[:, 2] * 3
    if int(ends.max()) > pix.numel() or int(meta[:, 1:].min()) < 1:
        raise ValueError("malformed pixel table")
    res = {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in batch.items()
           if k not in ("pixels", "pixel_meta")}
    dev = torch.device(device)
    pix_d = pix.to(dev, non_blocking=True) if dev.type == "cuda" else None   # the batch's ONE pixel copy
    if pix_d is not None and _ext.use_hip(pix_d):
        out = torch.empty((n, 3, out_h, out_w), dtype=torch.float32, device=dev)
        _ext.ext().resize_norm_u8(pix_d, meta.to(dev, non_blocking=True), out, list(IMAGENET_MEAN),
                                  list(IMAGENET_STD))
    else:
        ims = []
        for o, h, w in meta.tolist():
            x = pix[o:o + h * w * 3].view(h, w, 3).permute(2, 0, 1).unsqueeze(0).to(dev)
            ims.append(gpu_normalize_resize(x, out_h, out_w))
        out = torch.cat(ims)
    b = n // 2
    res["source_image"], res["target_image"] = out[:b], out[b:]
    return res

class PFPascalDataset(Dataset):
    """PF-Pascal keypoint pairs (lib/pf_dataset.py:11-112)."""

    def __init__(self, csv_file, dataset_path, output_size=(240, 240), transform=None, category=None,
                 pck_procedure="pf"):
        self.category_names = PF_CATEGORIES
        self.out_h, self.out_w = output_size
        pairs = pd.read_csv(csv_file)
        self.category = pairs.iloc[:, 2].to_numpy().astype("float")
        if category is not None:
            keep = np.nonzero(self.category == category)[0]
            self.category = self.category[keep]
            pairs = pairs.iloc[keep, :]
        self.pairs = pairs
        self.img_A_names = pairs.iloc[:, 0].tolist()
        self.img_B_names = pairs.iloc[:, 1].tolist()
        self.point_A_coords = pairs.iloc[:, 3:5]
        self.point_B_coords = pairs.iloc[:, 5:]
        self.dataset_path = dataset_path
        self.transform = transform
        self.pck_procedure = pck_procedure

    def __len__(self):
        return len(self.pairs)

    def get_image(self, name):
        image = read_image(os.path.join(self.dataset_path, name))
        im_size = torch.tensor(image.shape, dtype=torch.float32)
        return resize_bilinear(to_chw_float(image), self.out_h, self.out_w), im_size

    @staticmethod
    def parse_points(xs: str, ys: str, n: int = 20) -> torch.Tensor:
        x = np.array([float(v) for v in str(xs).split(";") if v != ""])
        y = np.array([float(v) for v in str(ys).split(";") if v != ""])
        out = -np.ones((2, n))
        out[0, : len(x)] = x
        out[1, : len(x)] = y
        return torch.tensor(out, dtype=torch.float32)

    def __getitem__(self, idx):
        image_a, size_a = self.get_image(self.img_A_names[idx])
        image_b, size_b = self.get_image(self.img_B_names[idx])
        pa = self.parse_points(self.point_A_coords.iloc[idx, 0], self.point_A_coords.iloc[idx, 1])
        pb = self.parse_points(self.point_B_coords.iloc[idx, 0], self.point_B_coords.iloc[idx, 1])
        n_pts = int(torch.sum(pa[0] != -1))
        if self.pck_procedure == "pf":
            l_pck = torch.tensor([float(torch.max(pa[:, :n_pts].max(1)[0] - pa[:, :n_pts].min(1)[0]))])
        elif self.pck_procedure == "scnet":
            pa[0, :n_pts] *= 224 / size_a[1]
            pa[1, :n_pts] *= 224 / size_a[0]
            pb[0, :n_pts] *= 224 / size_b[1]
            pb[1, :n_pts] *= 224 / size_b[0]
            size_a[0:2] = torch.tensor([224.0, 224.0])
            size_b[0:2] = torch.tensor([224.0, 224.0])
            l_pck = torch.tensor([224.0])
        else:
            raise ValueError(self.pck_procedure)
        sample = {"source_image": image_a, "target_image": image_b, "source_im_size": size_a,
                  "target_im_size": size_b, "source_points": pa, "target_points": pb, "L_pck": l_pck}
        if self.transform:
            sample = self.transform(sample)
        return sample


class SyntheticPairDataset(Dataset):
    """Random normalised image pairs of a fixed size (benchmarks, smoke tests)."""

    def __init__(self, length: int = 64, image_size=(400, 400), seed: int = 0):
        self.length = length
        self.h, self.w = image_size
        self.seed = seed

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 100003 + idx)
        a = torch.randn(3, self.h, self.w, generator=g)
        b = torch.randn(3, self.h, self.w, generator=g)
        size = torch.tensor([self.h, self.w, 3], dtype=torch.float32)
        return {"source_image": a, "target_image": b, "source_im_size": size, "target_im_size": size, "set": 0}


def synthetic_batch(batch: int, image_size=(400, 400), device="cpu", seed: int = 0):
    """One batch of random normalised pairs generated directly on ``device``."""
    g = torch.Generator(device=device).manual_seed(seed)
    h, w = image_size
    src = torch.randn(batch, 3, h, w, generator=g, device=device)
    tgt = torch.randn(batch, 3, h, w, generator=g, device=device)
    return {"source_image": src, "target_image": tgt}


def _smooth_texture(n: int, size: int, g: torch.Generator, device) -> torch.Tensor:
    """[n, 3, size, size] smooth random colour textures (sum of upsampled noise
    octaves), roughly ImageNet-normalised."""
    out = torch.zeros(n, 3, size, size, device=device)
    for cells, amp in ((6, 1.0), (12, 0.6), (24, 0.35), (48, 0.2)):
        noise = torch.randn(n, 3, cells, cells, generator=g, device=device)
        out += amp * torch.nn.functional.interpolate(noise, size=(size, size), mode="bicubic", align_corners=True)
    return out / out.flatten(1).std(1).view(n, 1, 1, 1)


def synthetic_correspondence_batch(batch: int, size: int, device="cpu", seed: int = 0, n_points: int = 20,
                                   max_shift: float = 0.15, max_rot_deg: float = 10.0, scale_range=(0.9, 1.1)):
    """Image pairs with a KNOWN dense correspondence (training-quality checks).

    A smooth texture is drawn on a 1.5x canvas; the source is its centre crop and
    the target samples the canvas through a random similarity transform
    (rotation, scale, shift), so target pixel p_t shows source pixel
    p_s = A (p_t - c) + c + t.  Keypoints are drawn in the target where p_s
    lands inside the source (PF-Pascal layout: [b, 2, n_points], -1 padded;
    ``L_pck`` = image size).  Everything is generated on ``device``."""
    g = torch.Generator(device=device).manual_seed(seed)
    canvas = int(round(1.5 * size))
    tex = _smooth_texture(batch, canvas, g, device)
    off = (canvas - size) / 2.0
    src = tex[:, :, int(off):int(off) + size, int(off):int(off) + size]
    u = lambda *s: torch.rand(*s, generator=g, device=device)  # noqa: E731
    ang = (u(batch) * 2 - 1) * max_rot_deg * 3.141592653589793 / 180
    sc = scale_range[0] + u(batch) * (scale_range[1] - scale_range[0])
    sh = (u(batch, 2) * 2 - 1) * max_shift * size
    A = torch.stack([torch.stack([sc * torch.cos(ang), -sc * torch.sin(ang)], -1),
                     torch.stack([sc * torch.sin(ang), sc * torch.cos(ang)], -1)], 1)      # [b, 2, 2] on (x, y)
    c = (size - 1) / 2.0
    ys, xs = torch.meshgrid(torch.arange(size, device=device, dtype=torch.float32),
                            torch.arange(size, device=device, dtype=torch.float32), indexing="ij")
    pt = torch.stack((xs, ys), -1).view(1, -1, 2) - c                                    # target pixels, centred
    ps = torch.einsum("bij,bnj->bni", A, pt.expand(batch, -1, -1)) + c + sh.view(batch, 1, 2)
    grid = (ps + off) / (canvas - 1) * 2 - 1                                               # canvas coords (align_corners)
    tgt = torch.nn.functional.grid_sample(tex, grid.view(batch, size, size, 2), mode="bilinear",
                                          padding_mode="border", align_corners=True)
    # keypoints: target points whose source correspondence is inside the source image
    cand = u(batch, 4 * n_points, 2) * (size - 1)
    cs = torch.einsum("bij,bnj->bni", A, cand - c) + c + sh.view(batch, 1, 2)
    ok = ((cs >= 0) & (cs <= size - 1)).all(-1)
    tp = torch.full((batch, 2, n_points), -1.0, device=device)
    sp = torch.full((batch, 2, n_points), -1.0, device=device)
    for i in range(batch):
        idx = torch.nonzero(ok[i]).view(-1)[:n_points]
        tp[i, :, :idx.numel()] = cand[i, idx].t()
        sp[i, :, :idx.numel()] = cs[i, idx].t()
    sz = torch.tensor([float(size), float(size), 3.0], device=device).expand(batch, 3)
    return {"source_image": src.contiguous(), "target_image": tgt.contiguous(), "source_points": sp,
            "target_points": tp, "source_im_size": sz, "target_im_size": sz,
            "L_pck": torch.full((batch, 1), float(size), device=device)}
