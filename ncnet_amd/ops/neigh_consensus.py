"""Symmetric NeighConsensus (stack of Conv4d + ReLU) as one autograd Function.

Reference semantics (lib/model.py:122-153): ``y = conv(x) + swap(conv(swap(x)))``
where ``conv`` is the Conv4d+ReLU stack and ``swap`` exchanges the A and B
axes of the correlation volume.  Because of the ReLUs this is not equivalent
to symmetrised filters, so both branches are computed.

MI355X design:
* both branches (and, in training, the positive and negative pairs) are one
  batch of volumes for every Conv4d launch: the swapped branch is built once
  as a bf16 transposed copy of the 1-channel input (0.8 MB per volume) instead
  of permuting the 16-channel activations;
* hidden activations are channels-last bf16 ``[V, I, J, K, L, 16]``; channel
  counts below 16 are zero-padded (zero weights and bias keep them at 0);
* bias + ReLU are fused into each conv's epilogue; the backward runs the
  data-gradient convs with the previous layer's ReLU mask fused into their
  epilogue, and the weight gradients with the MFMA wgrad kernels;
* ``y = z1 + z2^T`` (the branch un-swap) and, in backward, its transpose plus
  the last layer's ReLU mask are single tiled kernels.
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from . import _ext
from . import reference as ref
from .packing import (ij_groups, ij_in_grad, ij_in_weights, ij_out_grad, ij_out_weights, jc_in_grad, jc_in_weights,
                      jc_out_grad, jc_out_weights, kl_dgrad_in_weights, pack_kl_in, pack_kl_out, pack_w16,
                      pack_w16_planes, pack_w1in, pack_w1out, plane_dgrad_weights, transpose_for_dgrad)

HIP_KS = (3, 5)
# 1-channel layers through the j-offset channel encoding (csrc/jshift.hip) on
# the conv16 / wgrad16 kernels; NCNET_NC_JC=0 selects the dedicated
# 1-channel kernels (conv1in / conv1out / wgrad1) instead.
import os as _os

# Encoding of the 1-channel layers: "ij" (default: both plane offsets in
# channels, conv16 group-plane mode), "kl" (forward and data-gradient convs on
# the conv4d_kl.hip kernels, which resolve the in-plane (dk, dl) shifts in LDS
# -- no shifted copies or channel-planar partials in HBM; the weight gradients
# stay on the ij encoding; measured slower than ij at the 25^4 training shape:
# 37.1 vs 31.3 ms/step), "jc" (dj only), "direct" (conv1in / conv1out / wgrad1
# kernels).  NCNET_NC_JC=0 is the legacy spelling of "direct".
ENC = _os.environ.get("NCNET_NC_ENC", "ij")
if _os.environ.get("NCNET_NC_JC") == "0":
    ENC = "direct"
USE_JC = ENC == "jc"
USE_IJ = ENC in ("ij", "ijfull", "kl")
USE_KL = ENC == "kl"
# "ij" keeps the Cout=1 layer's forward and data gradient on the j encoding
# (one conv pass with an 8-channel fp32 output beats two group-plane passes
# with 16-channel planar outputs at 25^4: measured 1.97 vs 2.56 ms fwd) and
# uses the ij encoding for its weight gradient (plane-only wgrad, 1.5 vs
# 1.8 ms); "ijfull" runs that layer entirely on the ij encoding.  At KS = 3
# the ij encoding has a single group (one pass over one plane instead of 3
# planes), so it is used there in all modes.


def _out_ij_fwd(ks: int) -> bool:
    return ENC == "ijfull" or (ENC == "ij" and ks * ks <= 16)


# The Cout=1 layer's data gradient on the ij encoding: the group-plane conv
# reads ijpack(g, -1), which the weight gradient has already built, and
# writes the 16-channel masked gradient directly (no planar fp32 partials), so
# it replaces jpack + a KS-plane jc pass.  NCNET_NC_OUT_DGRAD=jc reverts.
OUT_DGRAD = _os.environ.get("NCNET_NC_OUT_DGRAD", "ij")


def _out_ij_dgrad(ks: int) -> bool:
    return _out_ij_fwd(ks) or (USE_IJ and OUT_DGRAD == "ij")
# wgrad16 kernel: 3 = sliding G-plane ring (default), 2 = 8-wave LDS-DMA per
# (di, dj) plane, 1 = 4-wave register-staged
WGRAD_VARIANT = int(_os.environ.get("NCNET_WGRAD_VARIANT", "3"))


def layer_kinds(channels, kernel_sizes):
    """Kernel family per layer or None if the stack needs the torch path."""
    kinds = []
    cin = 1
    for idx, (c, k) in enumerate(zip(channels, kernel_sizes)):
        if k not in HIP_KS or c > 16 or cin > 16:
            return None
        if cin == 1 and (c == 1 or idx > 0):
            return None
        if cin == 1:
            kinds.append("1in")
        elif c == 1:
            kinds.append("1out")
        else:
            kinds.append("16")
        cin = c
    if not kinds or kinds[-1] != "1out":
        return None
    return kinds


def wgrad_groups(ks: int, nitems: int) -> int:
    """Number of K-split groups of the wgrad kernels (~3000 workgroups for the
    KS*KS plane offsets; measured on MI355X: 120 groups at KS=5 beat 20 by 1.4x)."""
    env = _os.environ.get("NCNET_WGRAD_GROUPS")
    target = int(env) if env else 3072 // (ks * ks)
    return max(1, min(target, nitems))


def _std(w_ref: torch.Tensor) -> torch.Tensor:
    return ref.conv4d_weight_to_std(w_ref).float()


def _pad_bias(b: torch.Tensor, n: int) -> torch.Tensor:
    b = b.float()
    if b.numel() == n:
        return b.contiguous()
    out = b.new_zeros(n)
    out[: b.numel()] = b
    return out


def _stack_fwd(x0: torch.Tensor, ws, bs, kinds, save: list):
    """x0: [V,I,J,K,L] bf16 -> z fp32 [V,I,J,K,L]; appends layer inputs to save."""
    C = _ext.ext()
    h = x0
    V, I, J, K, L = x0.shape
    for li, (w_ref, b, kind) in enumerate(zip(ws, bs, kinds)):
        ks = w_ref.shape[0]
        w = _std(w_ref)
        save.append(h)
        last = li == len(kinds) - 1
        if kind == "1in" and USE_KL:
            # the backward ij-packs the saved 1-channel input for the weight gradient
            y = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.conv1to16_kl(h, pack_kl_in(w), _pad_bias(b, 16), None, y, ks, 1)
        elif kind == "1in" and USE_IJ:
            xs = torch.empty((ij_groups(ks), V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.ijpack(h, xs, ks, 1)
            save[-1] = xs  # the backward needs the ij-packed input
            y = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.conv16_fwd(xs, pack_w16_planes(ij_in_weights(w)), _pad_bias(b, 16), None, y, ks, 1, 0)
        elif kind == "1in" and USE_JC:
            xs = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.jpack(h, xs, ks, 1)
            save[-1] = xs  # the backward needs the j-packed input
            y = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.conv16_fwd(xs, pack_w16(jc_in_weights(w)), _pad_bias(b, 16), None, y, ks, 1, 1)
        elif kind == "1in":
            y = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.conv1in_fwd(h, pack_w1in(w), _pad_bias(b, 16), None, y, ks, 1)
        elif kind == "16":
            y = torch.empty((V, I, J, K, L, 16), dtype=torch.bfloat16, device=x0.device)
            C.conv16_fwd(h, pack_w16(w), _pad_bias(b, 16), None, y, ks, 1, 0)
        elif USE_KL:   # "1out"
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.conv16to1_kl(h, pack_kl_out(w), _pad_bias(b, 1), y, ks, 1, 1.0)
            if not last:
                y = y.to(torch.bfloat16)
        elif USE_IJ and _out_ij_fwd(ks):   # "1out"
            G = ij_groups(ks)
            wz = pack_w16_planes(ij_out_weights(w))
            nq = ks * ks
            z = torch.empty((nq, V, I, J, K, L), dtype=torch.float32, device=x0.device)   # planar by combo
            hx = h.unsqueeze(0)
            for gi in range(G):
                C.conv16_fwd(hx, wz[gi:gi + 1], None, None, z[16 * gi:min(nq, 16 * gi + 16)], ks, 4, 0)
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.ijsum(z, _pad_bias(b, 1), y, ks, 1, 1)
            del z
            if not last:
                y = y.to(torch.bfloat16)
        elif USE_JC or USE_IJ:
            z8 = torch.empty((ks, V, I, J, K, L), dtype=torch.float32, device=x0.device)   # planar, dj = 0..ks-1
            C.conv16_fwd(h, pack_w16(jc_out_weights(w)), None, None, z8, ks, 3, 1)
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.jsum(z8, _pad_bias(b, 1), y, ks, 1, 1)
            del z8
            if not last:
                y = y.to(torch.bfloat16)
        else:
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.conv1out_fwd(h, pack_w1out(w), _pad_bias(b, 1), y, ks, 1)
            if not last:
                y = y.to(torch.bfloat16)
        h = y
    return h


def wgrad_v3_ok(shape, ks: int) -> bool:
    """wgrad16v3 stages full-width X rows: L + ks - 1 <= 32."""
    return shape[4] + ks - 1 <= 32


def wgrad_v3_groups(shape, ks: int, dj_center: bool) -> int:
    """Column groups per dj for wgrad16v3: ~2 workgroups per CU in full mode
    (KS dj values), ~1 per CU in dj-centre mode, never more than the columns
    (v, j, tile).  Tile rule mirrors ncnet_wgrad16v3."""
    V, I, J, K, L = shape[:5]
    ntl = -(-(K * L) // 320)
    ncols = V * J * ntl
    target = 256 if dj_center else max(1, 512 // ks)
    env = _os.environ.get("NCNET_WGRAD_GROUPS")
    if env:
        target = int(env)
    return max(1, min(target, ncols))


def wgrad_plane_groups(nitems: int) -> int:
    """Groups of the plane-only wgrad (grid = groups): ~3 workgroups per CU."""
    env = _os.environ.get("NCNET_WGRAD_PLANE_GROUPS")
    return max(1, min(int(env) if env else 768, nitems))


def wgrad16_partials(C, x16: torch.Tensor, g16: torch.Tensor, ks: int, ng: int, dj_center):
    """Run the wgrad16 kernel and reduce its per-group partials.

    ``dj_center``: False/0 all (di, dj) plane offsets, True/1 dj = P only (j
    encoding), 2 only (P, P) (ij encoding, plane-only).  Returns (s, sb): s
    [dd, tap, ci, co], sb [16] = sum of g16 over all voxels (bias gradient,
    from the kernel's ones-MFMA in the centre block).  Variant 3 (sliding G
    ring) serves modes 0/1, variant 2 (8-wave LDS-DMA) mode 2 and volumes too
    wide for v3.
    """
    mode = int(dj_center)
    variant = WGRAD_VARIANT
    if mode == 2 or (variant == 3 and not wgrad_v3_ok(x16.shape, ks)):
        variant = 2
    if mode == 2:
        V, I, J, K, L = x16.shape[:5]
        ng = wgrad_plane_groups(V * I * J * ((K + 24) // 25) * ((L + 24) // 25))
    elif variant == 3:
        ng = wgrad_v3_groups(x16.shape, ks, bool(mode))
    rows = ng * (2 if variant >= 2 else 1)
    ndd = 1 if mode == 2 else (ks if mode else ks * ks)
    part = torch.empty((rows, ndd, ks * ks, 16, 16), dtype=torch.float32, device=x16.device)
    partb = torch.empty((rows, 16), dtype=torch.float32, device=x16.device)
    C.wgrad16(x16, g16, part, partb, ks, mode, variant)
    return part.sum(0), partb.sum(0)


def _reduce_wgrad16(s: torch.Tensor, ks: int, cout: int, cin: int) -> torch.Tensor:
    # s [dd, tap, ci, co] -> std [co, ci, di, dj, dk, dl]
    return s.permute(3, 2, 0, 1).reshape(16, 16, ks, ks, ks, ks)[:cout, :cin]


def _reduce_wgrad16_center(s: torch.Tensor, ks: int) -> torch.Tensor:
    # s [di, tap, ci, co] (dj = P only) -> [co, ci, di, dk, dl]
    return s.permute(3, 2, 0, 1).reshape(16, 16, ks, ks, ks)


def _reduce_wgrad1(part: torch.Tensor, ks: int, mode: int, c16: int) -> torch.Tensor:
    s = part.sum(0)  # [dd, tap, c16]
    if mode == 0:    # -> [co, 1, di, dj, dk, dl]
        return s.permute(2, 0, 1).reshape(16, 1, ks, ks, ks, ks)[:c16]
    # mode 1: tap index is flipped per (dk, dl): -> [1, ci, di, dj, dk, dl]
    s = s.reshape(ks, ks, ks, ks, 16).flip(2, 3)
    return s.permute(4, 0, 1, 2, 3).reshape(1, 16, ks, ks, ks, ks)[:, :c16]


# Weight gradients of the 16->16 and Cout=1 layers on a second HIP stream
# (NCNET_BWD_OVERLAP=0 disables): they depend only on the layer input and the
# incoming gradient, so wgrad(l) runs while the data-gradient chain continues
# on the main stream (dgrad(l) -> dgrad(l-1) -> ...).  The first layer's
# weight gradient stays on the main stream, which is idle by then.
BWD_OVERLAP = _os.environ.get("NCNET_BWD_OVERLAP", "1") == "1"
_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device):
    st = _SIDE_STREAMS.get(dev.index)
    if st is None:
        # NCNET_BWD_SIDE_PRIO=-1: high-priority side stream (tuning knob)
        st = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(
            device=dev, priority=int(_os.environ.get("NCNET_BWD_SIDE_PRIO", "0")))
    return st


class _OnSide:
    """Run a block on the side stream after everything queued on ``main``;
    inputs are marked in use by the side stream, outputs by ``main``."""

    def __init__(self, main, side, inputs):
        self.main, self.side, self.inputs = main, side, inputs
        self.ctx = None

    def __enter__(self):
        if self.side is None:
            return self
        self.side.wait_stream(self.main)
        for t in self.inputs:
            t.record_stream(self.side)
        self.ctx = torch.cuda.stream(self.side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


def _stack_bwd(g_last: torch.Tensor, saved, ws, kinds, channels, need_dx0: bool):
    """g_last: grad w.r.t. the last conv's PRE-activation (bf16, 1ch).
    Returns (dW list in checkpoint layout, db list, g_x0 fp32 or None)."""
    C = _ext.ext()
    nl = len(kinds)
    dws, dbs = [None] * nl, [None] * nl
    g = g_last
    gx0 = None
    main = side = None
    if BWD_OVERLAP and g_last.is_cuda:
        main = torch.cuda.current_stream(g_last.device)
        side = _side_stream(g_last.device)
    for li in range(nl - 1, -1, -1):
        kind, w_ref, h = kinds[li], ws[li], saved[li]
        ks = w_ref.shape[0]
        cout = channels[li]
        cin = 1 if li == 0 else channels[li - 1]
        w = _std(w_ref)
        V, I, J, K, L = h.shape[1:6] if h.dim() == 7 else h.shape[:5]
        nitems = V * I * J * ((K + 24) // 25) * ((L + 24) // 25)
        ng = wgrad_groups(ks, nitems)
        mask_prev = h if li > 0 else None   # ReLU output of the previous layer
        if kind == "1out" and USE_IJ:
            G = ij_groups(ks)
            gs = torch.empty((G,) + tuple(g.shape) + (16,), dtype=torch.bfloat16, device=h.device)
            C.ijpack(g, gs, ks, -1)                  # adjoint of ijsum
            with _OnSide(main, side, (h, gs)):
                parts = [wgrad16_partials(C, h, gs[gi], ks, ng, 2) for gi in range(G)]
                dw = ij_out_grad(torch.stack([p[0][0] for p in parts]), cin)
                qc = (ks // 2) * ks + ks // 2        # combo (P, P): its channel of ijpack(g, -1) is g itself
                db = parts[qc // 16][1][qc % 16].reshape(1)
                del parts
            if li > 0 or need_dx0:
                gi_ = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
                if USE_KL and mask_prev is not None:  # 1 -> Cin conv with flipped taps, ReLU mask fused
                    C.conv1to16_kl(g, pack_kl_in(kl_dgrad_in_weights(w)), None, mask_prev, gi_, ks, 2)
                elif _out_ij_dgrad(ks):              # reuses ijpack(g, -1) of the weight gradient
                    wd = pack_w16_planes(plane_dgrad_weights(ij_out_weights(w)))
                    C.conv16_fwd(gs, wd, None, mask_prev, gi_, ks, 2 if mask_prev is not None else 0, 0)
                else:                                # j encoding: 1 pass over the KS dj = P planes
                    del gs
                    gs = torch.empty(tuple(g.shape) + (16,), dtype=torch.bfloat16, device=h.device)
                    C.jpack(g, gs, ks, -1)
                    wt = transpose_for_dgrad(jc_out_weights(w))
                    C.conv16_fwd(gs, pack_w16(wt), None, mask_prev, gi_, ks, 2 if mask_prev is not None else 0, 1)
                g = gi_
                del gs
        elif kind == "1in" and USE_IJ:               # h is ijpack(X0) [G, ...] (kl: X0 itself)
            if h.dim() == 5:
                xs = torch.empty((ij_groups(ks),) + tuple(h.shape) + (16,), dtype=torch.bfloat16, device=h.device)
                C.ijpack(h, xs, ks, 1)
                h = xs
            G = h.shape[0]
            parts = [wgrad16_partials(C, h[gi], g, ks, ng, 2) for gi in range(G)]
            dw = ij_in_grad(torch.stack([p[0][0] for p in parts]), cout)
            db = parts[0][1][:cout]
            if li > 0:
                raise RuntimeError("internal: 1in layer must be first")
            if need_dx0:
                wd = pack_w16_planes(plane_dgrad_weights(ij_in_weights(w)))
                nq = ks * ks
                z = torch.empty((nq, V, I, J, K, L), dtype=torch.float32, device=h.device)
                gx = g.unsqueeze(0)
                for gi in range(G):
                    C.conv16_fwd(gx, wd[gi:gi + 1], None, None, z[16 * gi:min(nq, 16 * gi + 16)], ks, 4, 0)
                gx0 = torch.empty((V, I, J, K, L), dtype=torch.float32, device=h.device)
                C.ijsum(z, None, gx0, ks, 0, -1)      # adjoint of ijpack(+1)
        elif kind == "1out" and USE_JC:
            gs = torch.empty(tuple(g.shape) + (16,), dtype=torch.bfloat16, device=h.device)
            C.jpack(g, gs, ks, -1)                   # adjoint of jsum
            sw, sb = wgrad16_partials(C, h, gs, ks, ng, True)
            dw = jc_out_grad(_reduce_wgrad16_center(sw, ks), cin)
            db = sb[ks // 2].reshape(1)              # channel P of jpack(g, -1) is g itself
            if li > 0 or need_dx0:
                gi = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
                wt = transpose_for_dgrad(jc_out_weights(w))
                C.conv16_fwd(gs, pack_w16(wt), None, mask_prev, gi, ks, 2 if mask_prev is not None else 0, 1)
                g = gi
            del gs
        elif kind == "1in" and USE_JC:               # h is jpack(X0) (16ch)
            sw, sb = wgrad16_partials(C, h, g, ks, ng, True)
            dw = jc_in_grad(_reduce_wgrad16_center(sw, ks), cout)
            db = sb[:cout]
            if li > 0:
                raise RuntimeError("internal: 1in layer must be first")
            if need_dx0:
                z8 = torch.empty((ks,) + tuple(h.shape[:5]), dtype=torch.float32, device=h.device)
                wt = transpose_for_dgrad(jc_in_weights(w))
                C.conv16_fwd(g, pack_w16(wt), None, None, z8, ks, 3, 1)
                gx0 = torch.empty(tuple(h.shape[:5]), dtype=torch.float32, device=h.device)
                C.jsum(z8, None, gx0, ks, 0, -1)      # adjoint of jpack(+1)
        elif kind == "1out":
            if g.dim() == 6:
                raise RuntimeError("internal: 1out layer expects a 1-channel gradient")
            part = torch.empty((ng, ks * ks, ks * ks, 16), dtype=torch.float32, device=h.device)
            C.wgrad1(h, g, part, ks, 1, ng)
            dw = _reduce_wgrad1(part, ks, 1, cin)
            db = g.float().sum().reshape(1)
            if li > 0 or need_dx0:
                gi = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
                wt = transpose_for_dgrad(w)  # [16(ci as out), 1, k^4]
                C.conv1in_fwd(g, pack_w1in(wt), None, mask_prev, gi, ks, 2 if mask_prev is not None else 0)
                g = gi
        elif kind == "16":
            with _OnSide(main, side, (h, g)):
                sw, sb = wgrad16_partials(C, h, g, ks, ng, False)
                dw = _reduce_wgrad16(sw, ks, cout, cin)
                db = sb[:cout]
                del sw, sb
            if li > 0 or need_dx0:
                gi = torch.empty(h.shape, dtype=torch.bfloat16, device=h.device)
                wt = transpose_for_dgrad(w)
                C.conv16_fwd(g, pack_w16(wt), None, mask_prev, gi, ks, 2 if mask_prev is not None else 0, 0)
                g = gi
        else:  # "1in": h is the 1-channel input
            part = torch.empty((ng, ks * ks, ks * ks, 16), dtype=torch.float32, device=h.device)
            C.wgrad1(g, h, part, ks, 0, ng)
            dw = _reduce_wgrad1(part, ks, 0, cout)
            db = g.float().sum(dim=(0, 1, 2, 3, 4))[:cout]
            if li > 0:
                raise RuntimeError("internal: 1in layer must be first")
            if need_dx0:
                gi = torch.empty(h.shape, dtype=torch.float32, device=h.device)
                wt = transpose_for_dgrad(w)  # [1, 16, k^4]
                C.conv1out_fwd(g, pack_w1out(wt), None, gi, ks, 0)
                gx0 = gi
        dws[li] = dw
        dbs[li] = db
    if side is not None:
        main.wait_stream(side)
        for t in dws + dbs:          # produced on the side stream, consumed (and freed) on main
            t.record_stream(main)
    return [ref.conv4d_weight_from_std(d) for d in dws], dbs, gx0


def _swap_flat(x: torch.Tensor, shape_ab):
    """[V, I*J, K*L] -> [V, K*L, I*J] via the HIP tiled transpose."""
    C = _ext.ext()
    V = x.shape[0]
    i, j, k, l = shape_ab
    out = torch.empty((V, k * l, i * j), dtype=x.dtype, device=x.device)
    C.transpose(x.reshape(V, i * j, k * l), out)
    return out


class NeighConsensusFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, symmetric, kinds, channels, *params):
        ws, bs = params[0::2], params[1::2]
        V, _, I, J, K, L = x.shape
        R, Cc = I * J, K * L
        xb = x.reshape(V, I, J, K, L).to(torch.bfloat16).contiguous()
        saved_layers = []
        if symmetric:
            xt = _swap_flat(xb.reshape(V, R, Cc), (I, J, K, L)).reshape(V, K, L, I, J)
            if (I, J) == (K, L):
                x0 = torch.cat((xb, xt), 0)
                z = _stack_fwd(x0, ws, bs, kinds, saved_layers)
                branches = [saved_layers]
            else:
                s1, s2 = [], []
                z1 = _stack_fwd(xb, ws, bs, kinds, s1)
                z2 = _stack_fwd(xt, ws, bs, kinds, s2)
                z = torch.cat((z1.reshape(-1), z2.reshape(-1)))
                branches = [s1, s2]
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x.device)
            _ext.ext().combine_fwd(z, y, R, Cc)
        else:
            z = _stack_fwd(xb, ws, bs, kinds, saved_layers)
            branches = [saved_layers]
            y = z
        ctx.symmetric = symmetric
        ctx.kinds = kinds
        ctx.channels = channels
        ctx.dims = (V, I, J, K, L)
        ctx.nbranch = len(branches)
        flat = [t for br in branches for t in br]
        ctx.nper = len(branches[0])
        ctx.save_for_backward(z, *params, *flat)
        return y.reshape(V, 1, I, J, K, L)

    @staticmethod
    def backward(ctx, gy):
        z, *rest = ctx.saved_tensors
        nparam = 2 * len(ctx.kinds)
        params, flat = rest[:nparam], rest[nparam:]
        ws = params[0::2]
        V, I, J, K, L = ctx.dims
        R, Cc = I * J, K * L
        need_dx0 = ctx.needs_input_grad[0]
        gy = gy.reshape(V, R, Cc).float().contiguous()
        if ctx.symmetric:
            gz = torch.empty(z.numel(), dtype=torch.bfloat16, device=gy.device)
            _ext.ext().combine_bwd(gy, z, gz, R, Cc)
        else:
            gz = (gy.reshape(-1) * (z.reshape(-1) > 0)).to(torch.bfloat16)
        branches = [list(flat[b * ctx.nper:(b + 1) * ctx.nper]) for b in range(ctx.nbranch)]
        if ctx.nbranch == 1:
            nv = 2 * V if ctx.symmetric else V
            g_last = gz.reshape(nv, *((I, J, K, L)))
            dws, dbs, gx0 = _stack_bwd(g_last, branches[0], ws, ctx.kinds, ctx.channels, need_dx0)
        else:
            n1 = V * R * Cc
            g1 = gz[:n1].reshape(V, I, J, K, L)
            g2 = gz[n1:].reshape(V, K, L, I, J)
            dws1, dbs1, gxa = _stack_bwd(g1, branches[0], ws, ctx.kinds, ctx.channels, need_dx0)
            dws2, dbs2, gxb = _stack_bwd(g2, branches[1], ws, ctx.kinds, ctx.channels, need_dx0)
            dws = [a + b for a, b in zip(dws1, dws2)]
            dbs = [a + b for a, b in zip(dbs1, dbs2)]
            gx0 = None if gxa is None else torch.cat((gxa.reshape(-1), gxb.reshape(-1)))
        gx = None
        if need_dx0 and gx0 is not None:
            gx0 = gx0.reshape(-1)
            if ctx.symmetric:
                n1 = V * R * Cc
                ga = gx0[:n1].reshape(V, R, Cc)
                gb = _swap_flat(gx0[n1:].reshape(V, Cc, R), (K, L, I, J))
                gx = (ga + gb).reshape(V, 1, I, J, K, L)
            else:
                gx = gx0.reshape(V, 1, I, J, K, L)
        grads = []
        for dw, db in zip(dws, dbs):
            grads += [dw, db]
        return (gx, None, None, None, *grads)


# ---------------------------------------------------------------------------
# fp8 inference path (BASELINE config 5): OCP e4m3 activations and weights on
# the fp8 MFMA conv kernel, ij encoding for the 1-channel layers.

FP8 = torch.float8_e4m3fn


def _fp8_weights(packed_bf16: torch.Tensor):
    """Packed bf16 fragments -> (fp8 fragments scaled into the e4m3 range, 1/scale)."""
    amax = float(packed_bf16.abs().max())
    e = 0 if amax == 0 else int(np.floor(np.log2(240.0 / amax)))
    e = max(-8, min(12, e))
    return (packed_bf16.float() * 2.0 ** e).to(FP8), 2.0 ** -e


def _stack_fwd_fp8(x0: torch.Tensor, ws, bs, kinds) -> torch.Tensor:
    """x0 [V,I,J,K,L] bf16 -> last layer output fp32 [V,I,J,K,L] (ReLU'd), fp8 inside."""
    C = _ext.ext()
    V, I, J, K, L = x0.shape
    h = x0
    for li, (w_ref, b, kind) in enumerate(zip(ws, bs, kinds)):
        ks = w_ref.shape[0]
        w = _std(w_ref)
        if kind == "1in" and USE_KL:
            y = torch.empty((V, I, J, K, L, 16), dtype=FP8, device=x0.device)
            C.conv1to16_kl(h, pack_kl_in(w), _pad_bias(b, 16), None, y, ks, 1)
        elif kind == "1in":
            G = ij_groups(ks)
            xs = torch.empty((G, V, I, J, K, L, 16), dtype=FP8, device=x0.device)
            C.ijpack(h, xs, ks, 1)
            wq, osc = _fp8_weights(pack_w16_planes(ij_in_weights(w)))
            y = torch.empty((V, I, J, K, L, 16), dtype=FP8, device=x0.device)
            C.conv16f8_fwd(xs, wq, _pad_bias(b, 16), y, ks, 1, 0, osc)
        elif kind == "16":
            wq, osc = _fp8_weights(pack_w16(w))
            y = torch.empty((V, I, J, K, L, 16), dtype=FP8, device=x0.device)
            C.conv16f8_fwd(h, wq, _pad_bias(b, 16), y, ks, 1, 0, osc)
        elif USE_KL:  # "1out"
            wq, osc = _fp8_weights(pack_kl_out(w))
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.conv16to1_kl(h, wq, _pad_bias(b, 1), y, ks, 1, osc)
            if li != len(kinds) - 1:
                raise RuntimeError("fp8 NC path: the 1-channel output layer must be last")
        else:  # "1out"
            G, nq = ij_groups(ks), ks * ks
            wq, osc = _fp8_weights(pack_w16_planes(ij_out_weights(w)))
            z = torch.empty((nq, V, I, J, K, L), dtype=torch.float32, device=x0.device)
            hx = h.unsqueeze(0)
            for gi in range(G):
                C.conv16f8_fwd(hx, wq[gi:gi + 1], None, z[16 * gi:min(nq, 16 * gi + 16)], ks, 4, 0, osc)
            y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x0.device)
            C.ijsum(z, _pad_bias(b, 1), y, ks, 1, 1)
            del z
            if li != len(kinds) - 1:
                raise RuntimeError("fp8 NC path: the 1-channel output layer must be last")
        h = y
    return h


def neigh_consensus_fp8(x: torch.Tensor, weights, biases, kinds, symmetric: bool = True) -> torch.Tensor:
    """Inference-only NeighConsensus with fp8 operands (no autograd)."""
    V, _, I, J, K, L = x.shape
    R, Cc = I * J, K * L
    xb = x.reshape(V, I, J, K, L).to(torch.bfloat16).contiguous()
    if not symmetric:
        return _stack_fwd_fp8(xb, weights, biases, kinds).reshape(V, 1, I, J, K, L)
    xt = _swap_flat(xb.reshape(V, R, Cc), (I, J, K, L)).reshape(V, K, L, I, J)
    if (I, J) == (K, L):
        z = _stack_fwd_fp8(torch.cat((xb, xt), 0), weights, biases, kinds)
    else:
        z = torch.cat((_stack_fwd_fp8(xb, weights, biases, kinds).reshape(-1),
                       _stack_fwd_fp8(xt, weights, biases, kinds).reshape(-1)))
    y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x.device)
    _ext.ext().combine_fwd(z, y, R, Cc)
    return y.reshape(V, 1, I, J, K, L)


# ---------------------------------------------------------------------------
# Fused InLoc NC (csrc/nc_fused.hip): kernel sizes (3, 3), channels (<=16, 1),
# inference.  The hidden activation stays in LDS; HBM sees the input and the
# output volume once.  NCNET_NC_FUSED=0 falls back to the layer-by-layer path.
FUSED = _os.environ.get("NCNET_NC_FUSED", "1") != "0"
_FUSED_LDS = 78 * 1024          # two workgroups per CU (160 KB LDS)


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


@functools.lru_cache(maxsize=64)
def fused_tiles(V: int, I: int, J: int, K: int, L: int):
    """(TK, TL, R, IR) of nc_fused_k3: a (k, l) tile within the kernel's limits
    ((TK+2)(TL+2) <= 512, TK*TL <= 384, (TK+4)(TL+4) <= 512) minimising the
    padded layer-1 + layer-2 work, then R output planes per workgroup (as many
    as the LDS ring allows) and row segments of IR rows until the grid has
    ~2 workgroups per CU."""
    best = None
    for tk in range(1, min(K, 28) + 1):
        for tl in range(1, min(L, 28) + 1):
            if (tk + 2) * (tl + 2) > 512 or tk * tl > 384 or (tk + 4) * (tl + 4) > 512:
                continue
            n = _cdiv(K, tk) * _cdiv(L, tl)
            cost = n * (_cdiv((tk + 2) * (tl + 2), 16) + _cdiv(tk * tl, 16))
            if best is None or cost < best[0]:
                best = (cost, tk, tl)
    _, tk, tl = best
    fixed = (tk + 4) * (tl + 10) * 32 + (tk + 2) * (tl + 8) * 32 + 2 * 5 * 64 * 16
    r_max = max(1, (_FUSED_LDS - fixed) // (12 * tk * tl))
    base = V * _cdiv(K, tk) * _cdiv(L, tl)

    def nwg(r, ir):
        return base * _cdiv(J, r) * _cdiv(I, ir)

    # the kernel is latency-bound (two barriers per hidden plane): prefer >= ~500
    # workgroups (two per CU), first by splitting rows (halo (IR+2)/IR), then
    # planes ((R+2)/R).  Measured at 3200 px: 500 workgroups (R=10, IR=75)
    # 4.3 ms vs 6.4 ms for 1000 (IR=37); at 1600 px R=4, IR=5 0.55 ms.
    R, IR = min(J, r_max), I
    while nwg(R, IR) < 500 and IR > 5:
        IR = max(5, IR // 2)
    while nwg(R, IR) < 500 and R > 4:
        R -= 1
    return tk, tl, R, IR


def _fused_weights(weights, biases):
    w1, w2 = _std(weights[0]), _std(weights[1])
    W1p = pack_w16_planes(ij_in_weights(w1))[0].contiguous()
    W2p = pack_w16_planes(ij_out_weights(w2))[0].contiguous()
    return W1p, _pad_bias(biases[0], 16), W2p, _pad_bias(biases[1], 1)


def _run_fused(xb: torch.Tensor, wts) -> torch.Tensor:
    V, I, J, K, L = xb.shape
    y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=xb.device)
    tk, tl, R, IR = fused_tiles(V, I, J, K, L)
    _ext.ext().nc_fused_k3(xb, *wts, y, R, IR, tk, tl)
    return y


def neigh_consensus_fused(x: torch.Tensor, weights, biases, symmetric: bool = True) -> torch.Tensor:
    """Inference NeighConsensus of a (3, 3) / (<=16, 1) stack on the fused kernel."""
    V, _, I, J, K, L = x.shape
    R, Cc = I * J, K * L
    wts = _fused_weights(weights, biases)
    xb = x.reshape(V, I, J, K, L).to(torch.bfloat16).contiguous()
    if not symmetric:
        return _run_fused(xb, wts).reshape(V, 1, I, J, K, L)
    xt = _swap_flat(xb.reshape(V, R, Cc), (I, J, K, L)).reshape(V, K, L, I, J)
    if (I, J) == (K, L):
        z = _run_fused(torch.cat((xb, xt), 0), wts)
    else:
        z = torch.cat((_run_fused(xb, wts).reshape(-1), _run_fused(xt, wts).reshape(-1)))
    y = torch.empty((V, I, J, K, L), dtype=torch.float32, device=x.device)
    _ext.ext().combine_fwd(z, y, R, Cc)
    return y.reshape(V, 1, I, J, K, L)


def _fused_ok(kinds, kernel_sizes, x) -> bool:
    return (FUSED and not torch.is_grad_enabled() and list(kinds) == ["1in", "1out"]
            and list(kernel_sizes) == [3, 3] and x.shape[2] * x.shape[3] * x.shape[4] * x.shape[5] < 2 ** 31)


def neigh_consensus(x: torch.Tensor, weights, biases, channels, symmetric: bool = True, fp8: bool = False) -> torch.Tensor:
    """x: [V,1,I,J,K,L] fp32; weights in checkpoint layout [k, out, in, k, k, k].

    Inference of the InLoc (3,3)/(16,1) stack runs on the fused kernel (bf16
    operands, hidden layer kept on chip) whatever ``fp8`` says.  ``fp8``:
    inference of other 1-in/1-out stacks through the fp8 MFMA kernels (ignored
    when gradients are required or the stack shape has no fp8 kernels)."""
    kernel_sizes = [w.shape[0] for w in weights]
    kinds = layer_kinds(channels, kernel_sizes)
    if _ext.use_hip(x) and kinds is not None:
        if _fused_ok(kinds, kernel_sizes, x):
            return neigh_consensus_fused(x.float().contiguous(), weights, biases, symmetric)
        if fp8 and not torch.is_grad_enabled() and kinds[0] == "1in" and kinds[-1] == "1out":
            return neigh_consensus_fp8(x.float().contiguous(), weights, biases, kinds, symmetric)
        params = []
        for w, b in zip(weights, biases):
            params += [w, b]
        return NeighConsensusFn.apply(x.float().contiguous(), symmetric, tuple(kinds), tuple(channels), *params)
    return ref.neigh_consensus(x.float(), [w.float() for w in weights], [b.float() for b in biases], symmetric)
