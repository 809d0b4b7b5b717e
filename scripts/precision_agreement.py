#!/usr/bin/env python
"""Numerical agreement of the HIP inference precisions with the fp32 reference.

For synthetic pairs with a known correspondence (smooth textures under random
similarity warps) the same random-init model is evaluated by
* ``ref``  -- engine.reference_impl, the reference's fp32 computation
  (fp32 trunk, torch.bmm, per-slice conv3d NeighConsensus);
* ``bf16`` -- the default HIP path (bf16 operands, fp32 accumulation);
* ``fp16`` -- ``corr_dtype='fp16'``: bf16 trunk, IEEE-half features,
  correlation and NC on the f16 MFMA (the reference's half_precision; for
  PF-Pascal the 5,5,5 NC stays on the bf16 Conv4d kernels);
* ``fp32`` -- ``corr_dtype='fp32'``: fp32 trunk, bf16x3 correlation and NC;
* ``fp8``  -- ``corr_dtype='fp8'`` (InLoc config only): e4m3 correlation, bf16
  fused NC (the fp8 default);
* ``fp8_nc`` -- ``corr_dtype='fp8'`` with config ``nc_fp8``: e4m3 correlation
  and the e4m3 fused NC (BASELINE config 5 as specified).
Reported per precision: relative L2 of the output volume vs ``ref``, the
fraction of B cells (and A cells) whose best match (argmax over the other
image) equals the reference's, and PCK@0.1 of keypoint transfer.  Two
configurations: PF-Pascal (400 px, NC 5,5,5/16,16,1) and InLoc-style
(1600 px, relocalization k=2, NC 3,3/16,1).

    python scripts/precision_agreement.py --out profiles/r2_quality/precision_agreement.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd import config as _config  # noqa: E402
from ncnet_amd.data.datasets import synthetic_correspondence_batch  # noqa: E402
from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_inloc_forward  # noqa: E402
from ncnet_amd.eval.pck import pck  # noqa: E402
from ncnet_amd.eval.point_tnf import (PointsToPixelCoords, PointsToUnitCoords, bilinearInterpPointTnf,  # noqa: E402
                                      corr_to_matches)
from ncnet_amd.models import ImMatchNet  # noqa: E402


def agreement(c, r):
    V = c.shape[0]
    i, j, k, l = c.shape[2:]
    c3, r3 = c.reshape(V, i * j, k * l).float(), r.reshape(V, i * j, k * l).float()
    b_agree = (c3.argmax(1) == r3.argmax(1)).float().mean().item()
    a_agree = (c3.argmax(2) == r3.argmax(2)).float().mean().item()
    rel = ((c3 - r3).norm() / r3.norm()).item()
    return {"rel_l2": rel, "argmax_agree_B": b_agree, "argmax_agree_A": a_agree}


def pck_batch(corr, b, delta=None, k=1):
    matches = corr_to_matches(corr, delta4d=delta, k_size=k, do_softmax=True)[:4]
    tn = PointsToUnitCoords(b["target_points"], b["target_im_size"])
    warped = PointsToPixelCoords(bilinearInterpPointTnf(matches, tn), b["source_im_size"])
    v = pck(b["source_points"], warped, b["L_pck"].view(-1), 0.1)
    return v[~torch.isnan(v)].tolist()


def run_cfg(name, size, ks, ch, k_reloc, nbatch, batch, precisions, dev):
    torch.manual_seed(0)
    model = ImMatchNet(ncons_kernel_sizes=ks, ncons_channels=ch, relocalization_k_size=k_reloc).to(dev).eval()
    for p in model.NeighConsensus.parameters():          # populated ReLU pattern
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.1)
    alg = ReferenceAlgorithm(model, torch.float32)
    out = {p: {"rel_l2": [], "argmax_agree_B": [], "argmax_agree_A": [], "pck": []} for p in precisions}
    out["ref"] = {"pck": []}
    with torch.inference_mode():
        for it in range(nbatch):
            b = synthetic_correspondence_batch(batch, size, dev, seed=500 + it)
            if k_reloc > 1:
                r, rdelta = reference_inloc_forward(alg, b["source_image"], b["target_image"], k_reloc,
                                                    nc_dtype=torch.float32)
                r = r.float()
            else:
                r, rdelta = alg(b), None
            out["ref"]["pck"] += pck_batch(r, b, rdelta, max(1, k_reloc))
            for p in precisions:
                model.corr_dtype = "fp8" if p == "fp8_nc" else p
                model.compute_dtype = torch.float32 if p == "fp32" else torch.bfloat16
                with _config.override(nc_fp8=p == "fp8_nc"):
                    res = model(b)
                c, delta = (res if k_reloc > 1 else (res, None))
                a = agreement(c, r)
                for kk, vv in a.items():
                    out[p][kk].append(vv)
                out[p]["pck"] += pck_batch(c, b, delta, max(1, k_reloc))
    summ = {}
    for p, d in out.items():
        summ[p] = {kk: (sum(vv) / len(vv) if vv else None) for kk, vv in d.items()}
    return {"config": {"name": name, "image_size": size, "ncons_kernel_sizes": ks, "ncons_channels": ch,
                       "relocalization_k_size": k_reloc, "pairs": nbatch * batch}, "summary": summ}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--pf-batches", type=int, default=4)
    ap.add_argument("--inloc-batches", type=int, default=2)
    ap.add_argument("--inloc-sizes", type=int, nargs="+", default=[1600])
    a = ap.parse_args(argv)
    dev = torch.device("cuda")
    res = [run_cfg("pf_pascal_400", 400, [5, 5, 5], [16, 16, 1], 0, a.pf_batches, 4, ["bf16", "fp16", "fp32"], dev)]
    for size in a.inloc_sizes:
        res.append(run_cfg(f"inloc_{size}_k2", size, [3, 3], [16, 1], 2, a.inloc_batches, 1,
                           ["bf16", "fp16", "fp32", "fp8", "fp8_nc"], dev))
    for r in res:
        print(json.dumps(r), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
