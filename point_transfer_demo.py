#!/usr/bin/env python
"""Keypoint-transfer demo (the reference's point_transfer_demo.ipynb as a script).

Loads an NC-Net checkpoint (or random weights), draws a PF-Pascal test pair
(or a synthetic pair with --synthetic), computes matches with
corr_to_matches(do_softmax=True), transfers the target keypoints to the
source image with bilinearInterpPointTnf and saves a side-by-side figure.

    python point_transfer_demo.py --checkpoint trained_models/ncnet_pfpascal.pth.tar \
        --eval_dataset_path datasets/pf-pascal/ --out demo.png
    python point_transfer_demo.py --synthetic --out demo.png      # no dataset / weights
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.data import NormalizeImageDict, PFPascalDataset  # noqa: E402
from ncnet_amd.data.transforms import normalize_image  # noqa: E402
from ncnet_amd.eval.pck import pck  # noqa: E402
from ncnet_amd.eval.point_tnf import (PointsToPixelCoords, PointsToUnitCoords, bilinearInterpPointTnf,  # noqa: E402
                                      corr_to_matches)
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.utils.plot import plot_image  # noqa: E402


def synthetic_pair(size: int, seed: int = 0):
    """A smooth random image and a shifted copy, keypoints moved by the same shift."""
    g = torch.Generator().manual_seed(seed)
    base = torch.nn.functional.interpolate(torch.rand(1, 3, 12, 12, generator=g), size=(size + 40, size + 40),
                                           mode="bilinear", align_corners=True)[0]
    dy, dx = 17, 23
    src = base[:, :size, :size]
    tgt = base[:, dy:dy + size, dx:dx + size]
    tp = torch.full((2, 20), -1.0)
    tp[:, :8] = torch.rand(2, 8, generator=g) * (size - 80) + 40
    sp = tp.clone()
    sp[0, :8] += dx
    sp[1, :8] += dy
    sz = torch.tensor([float(size), float(size), 3.0])
    return {"source_image": normalize_image(src)[None], "target_image": normalize_image(tgt)[None],
            "source_points": sp[None], "target_points": tp[None], "source_im_size": sz[None],
            "target_im_size": sz[None], "L_pck": torch.tensor([[float(size)]])}


def main(argv=None):
    ap = argparse.ArgumentParser(description="NC-Net keypoint transfer demo")
    ap.add_argument("--checkpoint", type=str, default="")
    ap.add_argument("--eval_dataset_path", type=str, default="datasets/pf-pascal/")
    ap.add_argument("--image_size", type=int, default=400)
    ap.add_argument("--pair", type=int, default=-1, help="test pair index (default: random)")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--out", type=str, default="point_transfer_demo.png")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = ImMatchNet(use_cuda=dev.type == "cuda", checkpoint=a.checkpoint or None,
                       ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(dev).eval()
    if a.synthetic:
        batch = synthetic_pair(a.image_size, a.seed)
    else:
        ds = PFPascalDataset(csv_file=os.path.join(a.eval_dataset_path, "image_pairs/test_pairs.csv"),
                             dataset_path=a.eval_dataset_path,
                             transform=NormalizeImageDict(["source_image", "target_image"]),
                             output_size=(a.image_size, a.image_size), pck_procedure="scnet")
        idx = a.pair if a.pair >= 0 else int(np.random.default_rng(a.seed).integers(len(ds)))
        batch = {k: (v[None] if torch.is_tensor(v) else v) for k, v in ds[idx].items()}
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in batch.items()}
    with torch.inference_mode():
        corr4d = model(batch)
        xA, yA, xB, yB, score = corr_to_matches(corr4d, do_softmax=True)
        tnorm = PointsToUnitCoords(batch["target_points"], batch["target_im_size"])
        warped = PointsToPixelCoords(bilinearInterpPointTnf((xA, yA, xB, yB), tnorm), batch["source_im_size"])
        acc = pck(batch["source_points"], warped, batch["L_pck"].view(-1).float())
    valid = batch["target_points"][0, 0] != -1
    print(f"PCK@0.1 of this pair: {float(acc[0]):.3f} ({int(valid.sum())} keypoints)")

    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    # points are in original-image pixels; scale to the resized display images
    def disp(points, im_size):
        h, w = float(im_size[0, 0]), float(im_size[0, 1])
        p = points[0, :, valid].detach().cpu().numpy().copy()
        p[0] *= a.image_size / w
        p[1] *= a.image_size / h
        return p

    fig, ax = plt.subplots(1, 2, figsize=(10, 5))
    ax[0].imshow(plot_image(batch["target_image"], return_im=True))
    tp = disp(batch["target_points"], batch["target_im_size"])
    ax[0].scatter(tp[0], tp[1], c=np.arange(tp.shape[1]), cmap="tab20", s=40)
    ax[0].set_title("target keypoints")
    ax[1].imshow(plot_image(batch["source_image"], return_im=True))
    wp = disp(warped, batch["source_im_size"])
    sp = disp(batch["source_points"], batch["source_im_size"])
    ax[1].scatter(sp[0], sp[1], c=np.arange(sp.shape[1]), cmap="tab20", s=40, marker="x")
    ax[1].scatter(wp[0], wp[1], c=np.arange(wp.shape[1]), cmap="tab20", s=40)
    ax[1].set_title("transferred (o) vs ground truth (x)")
    for x in ax:
        x.set_axis_off()
    fig.savefig(a.out, bbox_inches="tight")
    print("saved " + a.out)
    return float(acc[0])


if __name__ == "__main__":
    main()
