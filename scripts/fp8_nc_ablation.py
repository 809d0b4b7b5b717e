#!/usr/bin/env python
"""Where the e4m3 NeighConsensus loses its argmax agreement (InLoc config).

The fused e4m3 NC (csrc/nc_fused.hip nc_fused_k3_f8) rounds three operands to
OCP e4m3: x0 (the mutual-matched, pooled correlation volume, scale sx), the
weights of both layers (scale sw = 2^e, amax -> 240) and the hidden 16-channel
activation (scale sh from a host-side worst-case bound).  This script runs the
InLoc forward of scripts/precision_agreement.py in fp32 up to x0, then the NC
emulated in fp32 with any subset of those roundings (and hi/lo splits or other
scales), followed by MutualMatching, and reports the argmax agreement with the
unrounded fp32 NC.  It isolates the NC's share of the error from the
correlation's.

    python scripts/fp8_nc_ablation.py [--size 1600] [--pairs 2] [--out f.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd.data.datasets import synthetic_correspondence_batch  # noqa: E402
from ncnet_amd.engine.reference_impl import ReferenceAlgorithm  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.ops import reference as ref  # noqa: E402
from ncnet_amd.ops.neigh_consensus import FP8_NC_X_SCALE, _pow2_scale  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from precision_agreement import agreement  # noqa: E402

E4M3 = torch.float8_e4m3fn


def q8(t, s):
    """e4m3 rounding at scale s, returned unscaled in fp32."""
    return (t * s).clamp(-448, 448).to(E4M3).float() / s


def q8_split(t, s, hi_lo):
    """hi (+ lo: the e4m3 rounding of the residual, at 16x the scale)."""
    h = q8(t, s)
    return h + q8(t - h, s * 16) if hi_lo else h


def emulate(x0, w1, b1, w2, b2, qx=False, qw=False, qh=False, x_lo=False, h_lo=False, w_lo=False,
            sh_mode="bound", dtype=None):
    """Symmetric 2-layer NC in fp32 with the chosen roundings; dtype=bf16 rounds
    the same operands to bf16 instead (the bf16 fused kernel)."""
    sx = FP8_NC_X_SCALE
    sw1 = _pow2_scale(float(w1.abs().max()), 240.0)
    sw2 = _pow2_scale(float(w2.abs().max()), 240.0)
    hb = float((w1.abs().flatten(1).sum(1) + b1.clamp(min=0)).max())
    rq = (lambda t, s, lo: t.to(dtype).float()) if dtype is not None else q8_split
    W1 = rq(w1, sw1, w_lo) if qw else w1
    W2 = rq(w2, sw2, w_lo) if qw else w2

    def stack(v):
        v = rq(v, sx, x_lo) if qx else v
        h = F.relu(ref.conv4d(v, ref.conv4d_weight_from_std(W1), b1))
        if qh:
            if sh_mode == "bound":
                sh = _pow2_scale(hb, 440.0)
            else:                                   # calibrated on this volume's hidden amax
                sh = _pow2_scale(float(h.abs().max()), 440.0)
            h = rq(h, sh, h_lo)
        return F.relu(ref.conv4d(h, ref.conv4d_weight_from_std(W2), b2))
    return stack(x0) + ref.swap_ab(stack(ref.swap_ab(x0)))


VARIANTS = {
    "none": {},
    "bf16_all": dict(qx=True, qw=True, qh=True, dtype=torch.bfloat16),
    "e4m3_x": dict(qx=True),
    "e4m3_w": dict(qw=True),
    "e4m3_h": dict(qh=True),
    "e4m3_all": dict(qx=True, qw=True, qh=True),
    "e4m3_all_h_calibrated": dict(qx=True, qw=True, qh=True, sh_mode="amax"),
    "e4m3_all_x_hilo": dict(qx=True, qw=True, qh=True, x_lo=True),
    "e4m3_all_w_hilo": dict(qx=True, qw=True, qh=True, w_lo=True),
    "e4m3_all_h_hilo": dict(qx=True, qw=True, qh=True, h_lo=True),
    "e4m3_all_xw_hilo": dict(qx=True, qw=True, qh=True, x_lo=True, w_lo=True),
    "e4m3_all_xh_hilo": dict(qx=True, qw=True, qh=True, x_lo=True, h_lo=True),
}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1600)
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--out", type=str, default="")
    a = ap.parse_args(argv)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], relocalization_k_size=2).to(dev).eval()
    for p in model.NeighConsensus.parameters():          # as precision_agreement.py: populated ReLU pattern
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.1)
    alg = ReferenceAlgorithm(model, torch.float32)
    layers = model.NeighConsensus.conv_layers()
    # checkpoint layout [k, out, in, k, k, k] -> [out, in, k, k, k, k]
    w1, w2 = (l.weight_ref().float().permute(1, 2, 0, 3, 4, 5).contiguous() for l in layers)
    b1, b2 = (l.bias.float() for l in layers)
    res = {k: {"argmax_agree_B": [], "argmax_agree_A": [], "rel_l2": []} for k in VARIANTS}
    with torch.inference_mode():
        for it in range(a.pairs):
            b = synthetic_correspondence_batch(1, a.size, dev, seed=500 + it)
            fa, fb = alg._fe(b["source_image"]).float(), alg._fe(b["target_image"]).float()
            corr, _ = ref.maxpool4d(ref.correlation_4d(fa, fb), 2)
            x0 = ref.mutual_matching(corr)
            r = ref.mutual_matching(emulate(x0, w1, b1, w2, b2))
            for k, kw in VARIANTS.items():
                c = ref.mutual_matching(emulate(x0, w1, b1, w2, b2, **kw))
                for kk, vv in agreement(c, r).items():
                    res[k][kk].append(vv)
            print(f"pair {it}: x0 {tuple(x0.shape)}", flush=True)
    summ = {k: {kk: sum(v) / len(v) for kk, v in d.items()} for k, d in res.items()}
    for k, d in summ.items():
        print(f"{k:26s} B {100 * d['argmax_agree_B']:6.2f} %  A {100 * d['argmax_agree_A']:6.2f} %  "
              f"rel_l2 {d['rel_l2']:.2e}", flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"size": a.size, "pairs": a.pairs, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
