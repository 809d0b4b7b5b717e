#!/usr/bin/env python
"""Per-kernel timing at the headline-benchmark shapes.

Training step at per-GPU batch B=16: 2B volumes (pos + neg) x 2 symmetric
branches = 64 volumes of 25^4.  Prints ms per call and useful TFLOP/s
(2 * MACs of the mathematical op, not of padded/redundant MFMA work).

    python scripts/kbench.py [--vols 64] [--size 25] [--reps 10] [--only name,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ncnet_amd.ops import _ext  # noqa: E402
from ncnet_amd.ops.neigh_consensus import wgrad_groups  # noqa: E402
from ncnet_amd.ops.packing import (ij_groups, ij_in_weights, pack_w16, pack_w16_planes, pack_w1in,  # noqa: E402
                                   pack_w1out)


def with_env(key, val, fn):
    """Run fn with os.environ[key] = val (the launchers read their tuning switches per call)."""
    def run():
        old = os.environ.get(key)
        os.environ[key] = val
        try:
            fn()
        finally:
            if old is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = old
    return run


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vols", type=int, default=64)
    ap.add_argument("--size", type=int, default=25)
    ap.add_argument("--ks", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", type=str, default="")
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--json", type=str, default="")
    a = ap.parse_args()
    C = _ext.ext()
    V, S, ks = a.vols, a.size, a.ks
    dev = "cuda"
    shp = (V, S, S, S, S)
    nvox = V * S ** 4
    x16 = (torch.rand(shp + (16,), device=dev) * (torch.rand(shp + (16,), device=dev) > 0.5)).to(torch.bfloat16)
    x1 = torch.rand(shp, device=dev).to(torch.bfloat16)
    g16 = torch.randn(shp + (16,), device=dev).to(torch.bfloat16)
    g1 = torch.randn(shp, device=dev).to(torch.bfloat16)
    y16 = torch.empty_like(x16)
    y1 = torch.empty(shp, device=dev)
    b16 = torch.zeros(16, device=dev)
    b1 = torch.zeros(1, device=dev)
    w16 = pack_w16(torch.randn(16, 16, ks, ks, ks, ks, device=dev) * 0.05)
    w1i = pack_w1in(torch.randn(16, 1, ks, ks, ks, ks, device=dev) * 0.05)
    w1o = pack_w1out(torch.randn(1, 16, ks, ks, ks, ks, device=dev) * 0.05)
    ng = a.groups or wgrad_groups(ks, V * S * S)
    part16 = torch.empty((2 * ng, ks * ks, ks * ks, 16, 16), device=dev)
    partb = torch.empty((2 * ng, 16), device=dev)
    part1 = torch.empty((ng, ks * ks, ks * ks, 16), device=dev)
    part16c = torch.empty((2 * ng, ks, ks * ks, 16, 16), device=dev)
    z8 = torch.empty((ks,) + shp, device=dev)
    from ncnet_amd.ops.neigh_consensus import wgrad_v3_groups
    n3, n3c = wgrad_v3_groups(shp, ks, False), wgrad_v3_groups(shp, ks, True)
    p3 = torch.empty((2 * n3, ks ** 2, ks ** 2, 16, 16), device=dev)
    p3b = torch.empty((2 * n3, 16), device=dev)
    p3c = torch.empty((2 * n3c, ks, ks ** 2, 16, 16), device=dev)
    p3cb = torch.empty((2 * n3c, 16), device=dev)
    g16b = torch.empty_like(g16)
    # ij encoding of the 1-channel layers (the training path): ijpack + group-plane conv + plane-only wgrad
    G = ij_groups(ks)
    xs = torch.empty((G,) + shp + (16,), device=dev, dtype=torch.bfloat16)
    wij = pack_w16_planes(ij_in_weights(torch.randn(16, 1, ks, ks, ks, ks, device=dev) * 0.05))
    from ncnet_amd.ops.neigh_consensus import wgrad_plane_groups
    npg = wgrad_plane_groups(V * S * S * ((S + 24) // 25) ** 2)
    pp = torch.empty((2 * npg, 1, ks * ks, 16, 16), device=dev)
    ppb = torch.empty((2 * npg, 16), device=dev)
    taps = ks ** 4
    fl16 = 2.0 * nvox * taps * 256
    fl1 = 2.0 * nvox * taps * 16
    cases = {
        "conv16_fwd": (lambda: C.conv16_fwd(x16, w16, b16, None, y16, ks, 1, 0), fl16),
        "conv16_fwd_nt": (with_env("NCNET_NT_STORE", "1", lambda: C.conv16_fwd(x16, w16, b16, None, y16, ks, 1, 0)), fl16),
        "conv16_dgrad_mask": (lambda: C.conv16_fwd(g16, w16, None, x16, y16, ks, 2, 0), fl16),
        "conv16_center_f32": (lambda: C.conv16_fwd(x16, w16, None, None, z8, ks, 3, 1), fl16 / ks),
        "conv16_center_f32_nt": (with_env("NCNET_NT_STORE", "1", lambda: C.conv16_fwd(x16, w16, None, None, z8, ks, 3, 1)), fl16 / ks),
        "jpack": (lambda: C.jpack(x1, g16b, ks, 1), None),
        "jsum": (lambda: C.jsum(z8, b1, y1, ks, 1, 1), None),
        "conv1in_fwd": (lambda: C.conv1in_fwd(x1, w1i, b16, None, y16, ks, 1), fl1),
        "conv1in_dgrad_mask": (lambda: C.conv1in_fwd(g1, w1i, None, x16, y16, ks, 2), fl1),
        "conv1out_fwd": (lambda: C.conv1out_fwd(x16, w1o, b1, y1, ks, 1), fl1),
        "wgrad16": (lambda: C.wgrad16(x16, g16, part16[:ng], partb[:ng], ks, 0, 1), fl16),
        "wgrad16_center": (lambda: C.wgrad16(x16, g16, part16c[:ng], partb[:ng], ks, 1, 1), fl16 / ks),
        "wgrad16v2": (lambda: C.wgrad16(x16, g16, part16, partb, ks, 0, 2), fl16),
        "wgrad16v2_center": (lambda: C.wgrad16(x16, g16, part16c, partb, ks, 1, 2), fl16 / ks),
        "wgrad16v3": (lambda: C.wgrad16(x16, g16, p3, p3b, ks, 0, 3), fl16),
        "wgrad16v3_center": (lambda: C.wgrad16(x16, g16, p3c, p3cb, ks, 1, 3), fl16 / ks),
        "ijpack": (lambda: C.ijpack(x1, xs, ks, 1), None),
        "ijpack_v2": (with_env("NCNET_IJPACK_V", "2", lambda: C.ijpack(x1, xs, ks, 1)), None),
        "ijpack_v3": (with_env("NCNET_IJPACK_V", "3", lambda: C.ijpack(x1, xs, ks, 1)), None),
        "ijpack_v1": (with_env("NCNET_IJPACK_V", "1", lambda: C.ijpack(x1, xs, ks, 1)), None),
        "wgrad16v3_prio": (with_env("NCNET_WGRAD_FLAGS", "1", lambda: C.wgrad16(x16, g16, p3, p3b, ks, 0, 3)), fl16),
        "ij_1in_conv": (lambda: C.conv16_fwd(xs, wij, b16, None, y16, ks, 1, 0), fl1),
        "ij_1in_conv_nt": (with_env("NCNET_NT_STORE", "1", lambda: C.conv16_fwd(xs, wij, b16, None, y16, ks, 1, 0)), fl1),
        "ij_1in_conv_tpw1": (with_env("NCNET_GP_TPW", "1", lambda: C.conv16_fwd(xs, wij, b16, None, y16, ks, 1, 0)), fl1),
        "ij_out_dgrad": (lambda: C.conv16_fwd(xs, wij, None, x16, y16, ks, 2, 0), fl1),
        "ij_out_dgrad_nt": (with_env("NCNET_NT_STORE", "1", lambda: C.conv16_fwd(xs, wij, None, x16, y16, ks, 2, 0)), fl1),
        "ij_out_dgrad_tpw1": (with_env("NCNET_GP_TPW", "1", lambda: C.conv16_fwd(xs, wij, None, x16, y16, ks, 2, 0)), fl1),
        "wgrad16v2_plane": (lambda: C.wgrad16(xs[0], g16, pp, ppb, ks, 2, 2), fl1 / G),
        "wgrad1_mode0": (lambda: C.wgrad1(g16, x1, part1, ks, 0, ng), fl1),
        "wgrad1_mode1": (lambda: C.wgrad1(x16, g1, part1, ks, 1, ng), fl1),
    }
    only = set(a.only.split(",")) if a.only else None
    res = {}
    for name, (fn, fl) in cases.items():
        if only and name not in only:
            continue
        ms = timeit(fn, a.reps)
        tf = round(fl / ms / 1e9, 1) if fl else None
        res[name] = {"ms": round(ms, 4), "tflops": tf}
        print(f"{name:22s} {ms:9.3f} ms  " + (f"{tf:8.1f} TFLOP/s" if tf else ""), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"vols": V, "size": S, "ks": ks, "groups": ng, "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
