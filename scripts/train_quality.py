#!/usr/bin/env python
"""Training quality: the HIP bf16 trainer vs the fp32 reference algorithm.

Both start from the same random initialisation (ResNet-101 trunk with
re-estimated BatchNorm statistics, NC 5,5,5/16,16,1 with small positive
biases) and see the same batches of synthetic pairs with a KNOWN dense
correspondence (``data.datasets.synthetic_correspondence_batch``: smooth
textures, random similarity warps).  Run (a) is this framework's training step
(bf16 trunk plan, HIP correlation / MutualMatching / Conv4d kernels, FlatAdam),
run (b) is ``engine.reference_impl`` -- the reference's fp32 computation op for
op (per-slice conv3d Conv4d, torch.bmm, torch MutualMatching, train.py's weak
loss) with torch.optim.Adam.  Reported: both loss curves and keypoint-transfer
PCK@0.1 on held-out pairs (eval_pf_pascal.py's procedure: B->A matches with
softmax, bilinear transfer) before and after training.

    python scripts/train_quality.py --steps 200 --out profiles/r2_quality/train_quality.json
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd.data.datasets import synthetic_correspondence_batch  # noqa: E402
from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_weak_loss  # noqa: E402
from ncnet_amd.engine.trainer import make_adam, weak_loss  # noqa: E402
from ncnet_amd.eval.pck import pck  # noqa: E402
from ncnet_amd.eval.point_tnf import (PointsToPixelCoords, PointsToUnitCoords, bilinearInterpPointTnf,  # noqa: E402
                                      corr_to_matches)
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.ops import _ext  # noqa: E402
from ncnet_amd.ops import reference as ref  # noqa: E402


def pck_of(forward, pairs, alpha=0.1):
    vals = []
    with torch.no_grad():
        for b in pairs:
            corr = forward(b)
            matches = corr_to_matches(corr, do_softmax=True)[:4]
            tn = PointsToUnitCoords(b["target_points"], b["target_im_size"])
            warped = PointsToPixelCoords(bilinearInterpPointTnf(matches, tn), b["source_im_size"])
            vals.append(pck(b["source_points"], warped, b["L_pck"].view(-1), alpha))
    v = torch.cat(vals)
    return float(v[~torch.isnan(v)].mean())


def recalibrate_bn(model, size, dev, batches=4, batch=8):
    """No pretrained weights ship (no network): give the random-init trunk
    data-dependent BatchNorm statistics (running mean / var re-estimated on
    synthetic textures, weights untouched) so its frozen eval-mode features
    are normalised instead of dominated by one direction."""
    trunk = model.FeatureExtraction.model
    bns = [m for m in trunk.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for m in bns:
        m.reset_running_stats()
        m.momentum = None                       # cumulative average
    trunk.train()
    with torch.no_grad():
        for s in range(batches):
            b = synthetic_correspondence_batch(batch // 2, size, dev, seed=90_000 + s)
            trunk(torch.cat((b["source_image"], b["target_image"])))
    trunk.eval()
    model.FeatureExtraction._folded = None      # re-fold BN into the trunk plan


def run(args):
    dev = torch.device("cuda")
    torch.manual_seed(args.seed)
    m_h = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1],
                     feature_extraction_last_layer=args.last_layer).to(dev)
    recalibrate_bn(m_h, args.image_size, dev)
    # non-degenerate NC start: at the reference init (biases ~U(+-1/sqrt(fan_in))) a
    # negative last-layer bias on these weak random-trunk volumes zeroes the whole NC
    # output and its gradient; small positive biases keep both runs trainable
    for p in m_h.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.05)
    m_r = copy.deepcopy(m_h)
    if args.nc_precision == "fp32":      # fp32-accurate HIP training: bf16x3 correlation + NC
        m_h.nc_precision = "fp32"
        m_h.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[args.hip_trunk]
    elif args.nc_precision == "mixed":   # ImMatchNet(nc_precision='mixed'): bf16x3 trunk + NC forward
        m_h.nc_precision = "mixed"
        m_h.compute_dtype = torch.float32
        m_h.FeatureExtraction.fp32_trunk = "x3"
    if args.fp32_trunk:                  # 'x3' (bf16x3 plan) or 'miopen' (true fp32) for the fp32 trunk
        m_h.FeatureExtraction.fp32_trunk = args.fp32_trunk
    if getattr(args, "no_ref", False):
        return _run_hip_only(args, m_h, dev)
    rdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[args.ref_dtype]
    alg = ReferenceAlgorithm(m_r, rdt, conv=ref.conv4d)   # same sums as the reference, k conv3d per layer
    # fp16 autocast needs loss scaling (the weak loss is ~1e-8 in this regime)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 24) if args.ref_dtype == "fp16" else None
    p_h = [p for p in m_h.parameters() if p.requires_grad]
    p_r = [p for p in m_r.parameters() if p.requires_grad]
    opt_h = make_adam(p_h, args.lr)
    opt_r = torch.optim.Adam(p_r, lr=args.lr)
    eval_pairs = [synthetic_correspondence_batch(args.batch, args.image_size, dev, seed=10_000 + i)
                  for i in range(args.eval_batches)]
    fwd_h = lambda b: m_h(b)  # noqa: E731
    fwd_r = lambda b: alg(b)  # noqa: E731
    m_h.eval()
    m_r.eval()
    res = {"config": vars(args), "pck_init_hip": pck_of(fwd_h, eval_pairs), "pck_init_ref": pck_of(fwd_r, eval_pairs)}
    m_h.train()
    m_r.train()
    lh, lr_ = [], []
    t0 = time.time()
    for step in range(args.steps):
        batch = synthetic_correspondence_batch(args.batch, args.image_size, dev, seed=step)
        batch = {"source_image": batch["source_image"], "target_image": batch["target_image"]}
        opt_h.zero_grad(set_to_none=True)
        loss = weak_loss(m_h, batch)
        loss.backward()
        opt_h.step()
        opt_r.zero_grad(set_to_none=True)
        loss_r = reference_weak_loss(alg, batch)
        if scaler is None:
            loss_r.backward()
            opt_r.step()
        else:
            scaler.scale(loss_r).backward()
            scaler.step(opt_r)
            scaler.update()
        lh.append(float(loss.detach()))
        lr_.append(float(loss_r.detach()))
        if step % 5 == 0 or step == args.steps - 1:
            print(f"step {step}: hip {lh[-1]:.5f} ref {lr_[-1]:.5f} ({time.time() - t0:.0f}s)", flush=True)
    m_h.eval()
    m_r.eval()
    res.update({"loss_hip": lh, "loss_ref": lr_,
                "pck_final_hip": pck_of(fwd_h, eval_pairs), "pck_final_ref": pck_of(fwd_r, eval_pairs),
                "dispatch": dict(_ext.DISPATCH)})
    w = max(1, args.steps // 10)
    res["summary"] = {"loss_first_hip": float(np.mean(lh[:w])), "loss_last_hip": float(np.mean(lh[-w:])),
                      "loss_first_ref": float(np.mean(lr_[:w])), "loss_last_ref": float(np.mean(lr_[-w:])),
                      "window": w}
    return res


def _run_hip_only(args, m_h, dev):
    """The HIP run alone (precision ablations: scripts/precision_ablation.py):
    loss curve and PCK before / after, no reference run."""
    p_h = [p for p in m_h.parameters() if p.requires_grad]
    opt_h = make_adam(p_h, args.lr)
    eval_pairs = [synthetic_correspondence_batch(args.batch, args.image_size, dev, seed=10_000 + i)
                  for i in range(args.eval_batches)]
    fwd_h = lambda b: m_h(b)  # noqa: E731
    m_h.eval()
    res = {"config": vars(args), "pck_init_hip": pck_of(fwd_h, eval_pairs)}
    m_h.train()
    lh = []
    for step in range(args.steps):
        batch = synthetic_correspondence_batch(args.batch, args.image_size, dev, seed=step)
        batch = {"source_image": batch["source_image"], "target_image": batch["target_image"]}
        opt_h.zero_grad(set_to_none=True)
        loss = weak_loss(m_h, batch)
        loss.backward()
        opt_h.step()
        lh.append(float(loss.detach()))
    m_h.eval()
    res.update({"loss_hip": lh, "pck_final_hip": pck_of(fwd_h, eval_pairs)})
    w = max(1, args.steps // 10)
    res["summary"] = {"loss_first_hip": float(np.mean(lh[:w])), "loss_last_hip": float(np.mean(lh[-w:])), "window": w}
    return res


def _heartbeat(period=60):
    """MIOpen compiles its conv3d kernels (the reference run) on first use,
    minutes of silence on a fresh box: keep the log alive."""
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(period)
            print(f"[alive {time.time() - t0:.0f}s]", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main(argv=None):
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--image-size", type=int, default=320)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--eval-batches", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--last-layer", type=str, default="", help="trunk cut (default layer3, the reference's)")
    ap.add_argument("--nc-precision", choices=["bf16", "fp32", "mixed"], default="bf16",
                    help="HIP run's NeighConsensus precision (fp32: bf16x3 forward+backward)")
    ap.add_argument("--hip-trunk", choices=["bf16", "fp32"], default="fp32",
                    help="trunk dtype of the --nc-precision fp32 HIP run (the trunk is frozen)")
    ap.add_argument("--ref-dtype", choices=["fp32", "bf16", "fp16"], default="fp32",
                    help="the reference run's compute dtype (bf16 / fp16: autocast; fp16 with loss scaling)")
    ap.add_argument("--x3-drop", type=str, default="",
                    help="with --nc-precision fp32: comma list of bf16x3 stages run in plain bf16 "
                         "(ops/neigh_consensus.py X3_STAGES: corr, nc_in, nc_w, nc_act, nc_grad)")
    ap.add_argument("--no-ref", action="store_true", help="skip the fp32 reference run (ablations)")
    ap.add_argument("--fp32-trunk", choices=["", "x3", "miopen"], default="",
                    help="the fp32 trunk's implementation (default: the mode's own)")
    ap.add_argument("--out", type=str, default="")
    a = ap.parse_args(argv)
    from ncnet_amd.ops.neigh_consensus import x3_ablation
    with x3_ablation([x for x in a.x3_drop.split(",") if x]):
        res = run(a)
    print(json.dumps({k: v for k, v in res.items() if k not in ("loss_hip", "loss_ref")}))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)
    return res


if __name__ == "__main__":
    main()
