#!/usr/bin/env python
"""Localise nc_fused_k3_f8 errors: single-tap / single-combo weights through
each layer vs the fp64 stack on the same e4m3-rounded values."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ncnet_amd.ops import _ext  # noqa: E402
from ncnet_amd.ops import reference as ref  # noqa: E402

nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
DEV = "cuda"


def f8q(t, s):
    return (t.double() * s).float().clamp(-448, 448).to(torch.float8_e4m3fn).double() / s


def run(w1, w2, b1, b2, x0, cfg):
    ws = [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)]
    tens, (sx, inv1, sh, inv2) = nc._fused_weights_f8_build(ws, [b1, b2])
    sw1, sw2 = 1.0 / (inv1 * sx), 1.0 / (inv2 * sh)
    V, I, J, K, L = x0.shape
    y = torch.full(x0.shape, float("nan"), device=DEV)
    R, IR, tk, tl = cfg
    _ext.ext().nc_fused_k3_f8(x0, *tens, y, R, IR, tk, tl, sx, inv1, sh, inv2)
    torch.cuda.synchronize()
    xq = f8q(x0, sx).unsqueeze(1)
    h = torch.relu(ref.conv4d(xq, ref.conv4d_weight_from_std(f8q(w1, sw1))) + b1.double().view(1, -1, 1, 1, 1, 1))
    h = f8q(h, sh)
    yr = torch.relu(ref.conv4d(h, ref.conv4d_weight_from_std(f8q(w2, sw2))) + b2.double().view(1, -1, 1, 1, 1, 1))
    yr = yr.squeeze(1)
    e = float((y.double().cpu() - yr.cpu()).abs().max() / (yr.abs().max().cpu() + 1e-12))
    return e, float(y.abs().max()), float(yr.abs().max())


def main():
    torch.manual_seed(0)
    V, I, J, K, L = 1, 5, 6, 7, 9
    x0 = (torch.rand(V, I, J, K, L, device=DEV)).to(torch.bfloat16)
    cfg = (3, 3, 6, 7)
    b1, b2 = torch.zeros(16, device=DEV), torch.zeros(1, device=DEV)
    w2c = torch.zeros(1, 16, 3, 3, 3, 3, device=DEV)
    w2c[0, 0, 1, 1, 1, 1] = 1.0
    for c in (4, 0, 8):
        for t in range(9):
            w1 = torch.zeros(16, 1, 3, 3, 3, 3, device=DEV)
            w1[0, 0, c // 3, c % 3, t // 3, t % 3] = 1.0
            print("L1 combo", c, "tap", t, run(w1, w2c, b1, b2, x0, cfg), flush=True)
    w1c = torch.zeros(16, 1, 3, 3, 3, 3, device=DEV)
    w1c[:, 0, 1, 1, 1, 1] = 1.0
    for ch in (0, 5, 15):
        for c in (4, 0, 8, 2):
            for t in range(9):
                w2 = torch.zeros(1, 16, 3, 3, 3, 3, device=DEV)
                w2[0, ch, c // 3, c % 3, t // 3, t % 3] = 1.0
                print("L2 ch", ch, "combo", c, "tap", t, run(w1c, w2, b1, b2, x0, cfg), flush=True)


if __name__ == "__main__":
    main()
