#!/usr/bin/env python
"""PF-Pascal keypoint-transfer evaluation (reference CLI: eval_pf_pascal.py:27-30).

Flags as in the reference (--checkpoint, --image_size, --eval_dataset_path),
plus --batch_size (the reference only supports 1), --synthetic N (random
pairs with random keypoints, for smoke tests without the dataset) and
--ncons_* for checkpoint-less runs, and --precision bf16|fp16|fp32 (the
reference evaluates in fp32: eval_pf_pascal.py never halves; default bf16
here, fp32 = fp32 trunk + bf16x3 correlation and NeighConsensus, fp16 = bf16
trunk, IEEE-half features / correlation on the f16 MFMA, the NeighConsensus on
the bf16 Conv4d kernels).  Multi-GPU: pairs are sharded over ranks and the
per-pair PCK values are gathered on rank 0.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.data import NormalizeImageDict, PFPascalDataset  # noqa: E402
from ncnet_amd.eval.pck import pck_metric, summarize  # noqa: E402
from ncnet_amd.eval.point_tnf import corr_to_matches  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.parallel.dist import destroy, init_distributed  # noqa: E402


class SyntheticKeypointPairs(Dataset):
    def __init__(self, n, size):
        self.n, self.size = n, size

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(i)
        h, w = self.size
        pts = torch.full((2, 20), -1.0)
        pts[:, :10] = torch.rand(2, 10, generator=g) * 200 + 10
        sz = torch.tensor([224.0, 224.0, 3.0])
        return {"source_image": torch.randn(3, h, w, generator=g), "target_image": torch.randn(3, h, w, generator=g),
                "source_im_size": sz, "target_im_size": sz.clone(), "source_points": pts,
                "target_points": pts + torch.randn(2, 20, generator=g), "L_pck": torch.tensor([224.0])}


def main(argv=None):
    ap = argparse.ArgumentParser(description="Compute PF Pascal matches")
    ap.add_argument("--checkpoint", type=str, default="")
    ap.add_argument("--image_size", type=int, default=400)
    ap.add_argument("--eval_dataset_path", type=str, default="datasets/pf-pascal/", help="path to PF Pascal dataset")
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--ncons_kernel_sizes", nargs="+", type=int, default=[5, 5, 5])
    ap.add_argument("--ncons_channels", nargs="+", type=int, default=[16, 16, 1])
    ap.add_argument("--precision", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="bf16 (default), fp16 (IEEE-half features + correlation), fp32 (fp32-accurate: fp32 trunk, "
                         "bf16x3 correlation and NeighConsensus, the reference's numerics)")
    args = ap.parse_args(argv)
    ctx = init_distributed()
    if ctx.is_main:
        print("NC-Net evaluation script - PF Pascal dataset (ncnet_amd)")
    model = ImMatchNet(use_cuda=ctx.device.type == "cuda", checkpoint=args.checkpoint or None,
                       ncons_kernel_sizes=args.ncons_kernel_sizes, ncons_channels=args.ncons_channels,
                       dtype="fp32" if args.precision == "fp32" else "bf16", corr_dtype=args.precision).to(ctx.device)
    model.eval()
    size = (args.image_size, args.image_size)
    if args.synthetic:
        dataset = SyntheticKeypointPairs(args.synthetic, size)
    else:
        dataset = PFPascalDataset(csv_file=os.path.join(args.eval_dataset_path, "image_pairs/test_pairs.csv"),
                                  dataset_path=args.eval_dataset_path,
                                  transform=NormalizeImageDict(["source_image", "target_image"]), output_size=size,
                                  pck_procedure="scnet")
    idx = list(range(ctx.rank, len(dataset), ctx.world_size))
    loader = DataLoader(torch.utils.data.Subset(dataset, idx), batch_size=args.batch_size, shuffle=False)
    stats = {"point_tnf": {"pck": np.zeros((len(idx), 1))}}
    pos = 0
    with torch.inference_mode():
        for i, batch in enumerate(loader):
            batch = {k: (v.to(ctx.device) if torch.is_tensor(v) else v) for k, v in batch.items()}
            corr4d = model(batch)
            xA, yA, xB, yB, _ = corr_to_matches(corr4d, do_softmax=True)
            stats = pck_metric(batch, pos, (xA, yA, xB, yB), stats)
            pos += batch["source_image"].shape[0]
            if ctx.is_main:
                print(f"Batch: [{i}/{len(loader)} ({100.0 * i / max(1, len(loader)):.0f}%)]", flush=True)
    res = stats["point_tnf"]["pck"]
    if ctx.enabled:
        parts = [None] * ctx.world_size
        dist.all_gather_object(parts, res)
        res = np.concatenate(parts, 0)
        stats["point_tnf"]["pck"] = res
    if ctx.is_main:
        s = summarize(stats)
        print("Total: " + str(s["total"]))
        print("Valid: " + str(s["valid"]))
        print("PCK:", "{:.2%}".format(s["pck"]))
    destroy(ctx)
    return stats


if __name__ == "__main__":
    main()
