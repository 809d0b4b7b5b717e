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
from ncnet_amd.ops.neigh_consensus import wgrad_groups, wgrad_plane_groups, wgrad_v3_groups  # noqa: E402
from ncnet_amd.ops.packing import ij_groups, ij_in_weights, ij_out_weights, pack_w16, pack_w16_planes  # noqa: E402


_TUNING = {"NCNET_C1X_PD": "c1x_pd", "NCNET_CONV_V3": "conv_v3", "NCNET_WGRAD_V3": "wgrad_v3", "NCNET_GP_TPW": "gp_tpw",
           "NCNET_NT_STORE": "nt_store", "NCNET_WGRAD_FLAGS": "wgrad_flags"}


def with_env(key, val, fn):
    """Run fn with launcher tuning switch ``key`` (its NCNET_* name) set to val
    (config.override: the launchers never read the environment)."""
    def run():
        from ncnet_amd import config
        with config.override(**{_TUNING[key]: int(val)}):
            fn()
    return run


def _nc_fused_case(dev):
    """The InLoc 3200 px fused NeighConsensus (3,3 / 16,1) on one symmetric
    volume pair: [2, 75, 100, 75, 100] bf16 -> fp32."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    from ncnet_amd.ops import reference as ref
    g = torch.Generator(device=dev).manual_seed(5)
    x2 = torch.rand((2, 75, 100, 75, 100), device=dev, generator=g).to(torch.bfloat16)
    ws = [ref.conv4d_weight_from_std(torch.randn(16, 1, 3, 3, 3, 3, device=dev, generator=g) * 0.2),
          ref.conv4d_weight_from_std(torch.randn(1, 16, 3, 3, 3, 3, device=dev, generator=g) * 0.1)]
    bs = [torch.rand(16, device=dev, generator=g) * 0.1, torch.rand(1, device=dev, generator=g) * 0.1]
    return lambda: nc.neigh_consensus_fused_x2(x2, ws, bs)


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
    ap.add_argument("--rounds", type=int, default=1, help="repeat the selected cases (interleaved A/B)")
    ap.add_argument("--only", type=str, default="")
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
    y16 = torch.empty_like(x16)
    y1 = torch.empty(shp, device=dev)
    b16 = torch.zeros(16, device=dev)
    b1 = torch.zeros(1, device=dev)
    w16 = pack_w16(torch.randn(16, 16, ks, ks, ks, ks, device=dev) * 0.05)
    n3 = wgrad_v3_groups(shp, ks)
    p3 = torch.empty((2 * n3, ks ** 2, ks ** 2, 16, 16), device=dev)
    p3b = torch.empty((2 * n3, 16), device=dev)
    p3g = {n: (torch.empty((2 * n, ks ** 2, ks ** 2, 16, 16), device=dev), torch.empty((2 * n, 16), device=dev))
           for n in (51, 204, 306)}
    ng2 = wgrad_groups(ks, V * S * S * ((S + 24) // 25) ** 2)
    p2 = torch.empty((2 * ng2, ks ** 2, ks ** 2, 16, 16), device=dev)
    p2b = torch.empty((2 * ng2, 16), device=dev)
    # ij encoding of the 1-channel layers (the training path): ijpack + group-plane conv + plane-only wgrad
    G = ij_groups(ks)
    xs = torch.empty((G,) + shp + (16,), device=dev, dtype=torch.bfloat16)
    wij = pack_w16_planes(ij_in_weights(torch.randn(16, 1, ks, ks, ks, ks, device=dev) * 0.05))
    npg = wgrad_plane_groups(V * S * S * ((S + 24) // 25) ** 2)
    pp = torch.empty((2 * npg, 1, ks * ks, 16, 16), device=dev)
    ppb = torch.empty((2 * npg, 16), device=dev)
    wz = pack_w16_planes(ij_out_weights(torch.randn(1, 16, ks, ks, ks, ks, device=dev) * 0.05))
    from ncnet_amd.ops.packing import blk_out_weights
    wblk = pack_w16_planes(blk_out_weights(torch.randn(1, 16, ks, ks, ks, ks, device=dev) * 0.05))
    from ncnet_amd.ops.packing import cout1_taps_weights
    wct = cout1_taps_weights(torch.randn(1, 16, ks, ks, ks, ks, device=dev) * 0.05).to(torch.bfloat16)
    pq = torch.empty((1024, G, ks * ks, 16, 16), device=dev)
    pqb = torch.empty((1024, G, 16), device=dev)
    nq = ks * ks
    zq = torch.empty((nq,) + shp, device=dev)

    from ncnet_amd.ops.packing import pack_w1x
    lp, ppl = C.pad_geom(S, S, ks)
    xpad = torch.zeros((V * S * S, ppl), dtype=torch.bfloat16, device=dev)
    C.pad_planes(x1.reshape(V, S * S, S * S), xpad, S, S, ks, 0)
    w1x = pack_w1x(torch.randn(16, 1, ks, ks, ks, ks, device=dev) * 0.05)

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    p1x = torch.empty((ncu, ks * ks, 32, 16), device=dev)
    p1xb = torch.empty((ncu, 16), device=dev)

    def ij_out_fwd():
        for gi in range(G):
            C.conv16_fwd(x16.unsqueeze(0), wz[gi:gi + 1], None, None, zq[16 * gi:min(nq, 16 * gi + 16)], ks, 4)
        C.ijsum(zq, b1, y1, ks, 1, 1)
    taps = ks ** 4
    fl16 = 2.0 * nvox * taps * 256
    fl1 = 2.0 * nvox * taps * 16
    cases = {
        "conv16_fwd": (lambda: C.conv16_fwd(x16, w16, b16, None, y16, ks, 1), fl16),
        "conv16_dgrad_mask": (lambda: C.conv16_fwd(g16, w16, None, x16, y16, ks, 2), fl16),
        # same kernels with the other operand distribution (DVFS: the clock the
        # chip holds depends on the data, so fwd vs dgrad is compared both ways)
        "conv16_fwd_dense": (lambda: C.conv16_fwd(g16, w16, b16, None, y16, ks, 1), fl16),
        "conv16_dgrad_sparse": (lambda: C.conv16_fwd(x16, w16, None, x16, y16, ks, 2), fl16),
        "conv16_fwd_v3": (with_env("NCNET_CONV_V3", "1", lambda: C.conv16_fwd(x16, w16, b16, None, y16, ks, 1)), fl16),
        "conv16_dgrad_v3": (with_env("NCNET_CONV_V3", "1", lambda: C.conv16_fwd(g16, w16, None, x16, y16, ks, 2)), fl16),
        "conv16_f32": (lambda: C.conv16_fwd(x16, w16, None, None, torch.empty((16,) + shp, device=dev), ks, 4), fl16),
        "wgrad16v3": (lambda: C.wgrad16(x16, g16, p3, p3b, ks, 0, 3), fl16),
        "wgrad16v3_old": (with_env("NCNET_WGRAD_V3", "1", lambda: C.wgrad16(x16, g16, p3, p3b, ks, 0, 3)), fl16),
        "wgrad16v2": (lambda: C.wgrad16(x16, g16, p2, p2b, ks, 0, 2), fl16),
        **{f"wgrad16v3_g{n}": ((lambda n=n: C.wgrad16(x16, g16, p3g[n][0], p3g[n][1], ks, 0, 3)), fl16)
           for n in (51, 204, 306)},
        "wgrad16v3_prio": (with_env("NCNET_WGRAD_FLAGS", "1", lambda: C.wgrad16(x16, g16, p3, p3b, ks, 0, 3)), fl16),
        "ijpack": (lambda: C.ijpack(x1, xs, ks, 1), None),
        "pad_planes": (lambda: C.pad_planes(x1.reshape(V, S * S, S * S), xpad, S, S, ks, 0), None),
        "pad_planes_t": (lambda: C.pad_planes(x1.reshape(V, S * S, S * S), xpad, S, S, ks, 1), None),
        "nc_fused_3200": (_nc_fused_case(dev), 2.0 * 2 * (75 * 100) ** 2 * 2 * 16 * 81),
        "conv1x16_fwd": (lambda: C.conv1x16(xpad, w1x, b16, None, y16, ks, 1), fl1),
        "conv1x16_dgrad": (lambda: C.conv1x16(xpad, w1x, None, x16, y16, ks, 2), fl1),
        "conv1x16_fwd_pd2": (with_env("NCNET_C1X_PD", "2", lambda: C.conv1x16(xpad, w1x, b16, None, y16, ks, 1)), fl1),
        "conv1x16_dgrad_pd2": (with_env("NCNET_C1X_PD", "2", lambda: C.conv1x16(xpad, w1x, None, x16, y16, ks, 2)),
                               fl1),
        "conv1x16_fwd_pd3": (with_env("NCNET_C1X_PD", "3", lambda: C.conv1x16(xpad, w1x, b16, None, y16, ks, 1)), fl1),
        "conv1x16_dgrad_pd3": (with_env("NCNET_C1X_PD", "3", lambda: C.conv1x16(xpad, w1x, None, x16, y16, ks, 2)),
                               fl1),
        "wgrad1x16": (lambda: C.wgrad1x16(g16, xpad, p1x, p1xb, ks), fl1),
        "wgrad1x16_nobias": (lambda: C.wgrad1x16(x16, xpad, p1x, None, ks), fl1),
        "ij_1in_conv": (lambda: C.conv16_fwd(xs, wij, b16, None, y16, ks, 1), fl1),
        "ij_1in_conv_tpw1": (with_env("NCNET_GP_TPW", "1", lambda: C.conv16_fwd(xs, wij, b16, None, y16, ks, 1)), fl1),
        "ij_out_dgrad": (lambda: C.conv16_fwd(xs, wij, None, x16, y16, ks, 2), fl1),
        "ij_out_fwd_total": (ij_out_fwd, fl1),
        "ijsum": (lambda: C.ijsum(zq, b1, y1, ks, 1, 1), None),
        "blk_out_fwd": (lambda: C.conv16_blk_fwd(x16, wblk, b1, y1, ks, 1), fl1),
        "cout1_taps_fwd": (lambda: C.cout1_taps_fwd(x16, wct, b1, y1, ks, 1), fl1),
        "wgrad16v2_plane": (lambda: C.wgrad16(xs[0], g16, pp, ppb, ks, 2, 2), fl1 / G),
        "wgrad16p_1out": (lambda: C.wgrad16p(x16.unsqueeze(0), xs, pq, pqb, ks), fl1),
        "wgrad16p_1in": (lambda: C.wgrad16p(xs, g16.unsqueeze(0), pq, pqb, ks), fl1),
    }
    only = set(a.only.split(",")) if a.only else None
    res = {}
    for name, (fn, fl) in [kv for _ in range(a.rounds) for kv in cases.items()]:
        if only and name not in only:
            continue
        ms = timeit(fn, a.reps)
        tf = round(fl / ms / 1e9, 1) if fl else None
        res[name] = {"ms": round(ms, 4), "tflops": tf}
        print(f"{name:22s} {ms:9.3f} ms  " + (f"{tf:8.1f} TFLOP/s" if tf else ""), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"vols": V, "size": S, "ks": ks, "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
