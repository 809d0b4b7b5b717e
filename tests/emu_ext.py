"""A CPU stand-in for the HIP extension's Conv4d kernels (``ncnet_amd/_C.so``).

Each function has the binding's signature and buffer contract (packed MFMA
weight fragments in, bf16/fp32 buffers written in place) and computes the
kernel's math exactly in float64 from the packed operands: conv16_fwd
(full 4D or group-plane mode, epilogues 0/1/2/4), conv16_blk_fwd (output-plane
blocks of a Cout=1 layer), wgrad16 (full / plane-only
partial layout), ijpack / ijsum, combine and transpose.  It lets the CPU suite
check the Python orchestration of the HIP path (channel blocks, the ij
encoding, weight packing, symmetric branches, every gradient) against
autograd of the fp64 oracle, with bf16 rounding exactly where the GPU path
stores bf16.  The packed-weight decode inverts ``packing._idx16``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.packing import _idx16


def _unpack16(wp: torch.Tensor, ks: int) -> torch.Tensor:
    """[NPL, nq, 64, 8] packed fragments -> [NPL, 16 co, 16 ci, ks*ks taps] fp64."""
    co, ci, tap, valid = _idx16(ks)
    npl = wp.shape[0]
    w = torch.zeros(npl, 16, 16, ks * ks, dtype=torch.float64)
    src = wp.double()
    for pl in range(npl):
        w[pl, co[valid], ci[valid], tap[valid]] = src[pl][valid]
    return w


def _plane_conv(x, w, ks):
    """x [N, 16, K, L] fp64, w [16, 16, ks*ks] -> [N, 16, K, L] ("same" 2D conv)."""
    return F.conv2d(x, w.reshape(16, 16, ks, ks), padding=ks // 2)


def conv16_fwd(X, Wp, bias, M, Y, ks, epi):
    grp = X.dim() == 7
    xs = X.double()
    w = _unpack16(Wp, ks)
    if grp:
        G, V, I, J, K, L, _ = xs.shape
        acc = 0
        for s in range(G):
            xx = xs[s].permute(0, 1, 2, 5, 3, 4).reshape(V * I * J, 16, K, L)
            acc = acc + _plane_conv(xx, w[s], ks)
        out = acc.reshape(V, I, J, 16, K, L).permute(0, 1, 2, 4, 5, 3)      # [V,I,J,K,L,16]
    else:
        V, I, J, K, L, _ = xs.shape
        wstd = w.reshape(ks, ks, 16, 16, ks, ks).permute(2, 3, 0, 1, 4, 5)  # [co, ci, di, dj, dk, dl]
        out = ref.conv4d(xs.permute(0, 5, 1, 2, 3, 4), ref.conv4d_weight_from_std(wstd))
        out = out.permute(0, 2, 3, 4, 5, 1)
    if epi == 4:
        Y.copy_(out[..., :Y.shape[0]].permute(5, 0, 1, 2, 3, 4))
        return
    if epi == 1:
        out = torch.relu(out + bias.double())
    elif epi == 2:
        out = out * (M.double() > 0)
    Y.copy_(out)


def conv16_blk_fwd(X, Wp, bias, Y, ks, relu):
    """Output-plane-block Cout=1 conv: block (i0, j0) streams input planes
    (p, q) in [i0-P, i0+4+P) x [j0-P, j0+4+P); relative plane
    (p-i0+P)*(ks+3) + (q-j0+P) of the packed weights gives row r = 4a+b, i.e.
    output plane (i0+a, j0+b)."""
    xs = X.double()
    V, I, J, K, L, _ = xs.shape
    P, sp = ks // 2, ks + 3
    w = _unpack16(Wp, ks)                                     # [sp*sp, 16 rows, 16 ci, taps]
    acc = torch.zeros((V, I, J, K, L), dtype=torch.float64)
    for i0 in range(0, I, 4):
        for j0 in range(0, J, 4):
            for p in range(max(0, i0 - P), min(I, i0 + 4 + P)):
                for q in range(max(0, j0 - P), min(J, j0 + 4 + P)):
                    wp = w[(p - i0 + P) * sp + (q - j0 + P)]
                    rows = _plane_conv(xs[:, p, q].permute(0, 3, 1, 2), wp, ks)     # [V, 16 rows, K, L]
                    for r in range(16):
                        i, j = i0 + r // 4, j0 + r % 4
                        if i < I and j < J:
                            acc[:, i, j] += rows[:, r]
    if bias is not None:
        acc += float(bias.reshape(-1)[0])
    Y.copy_(torch.relu(acc) if relu else acc)


def wgrad16(X, G, part, partb, ks, mode, variant):
    with torch.enable_grad():      # called from inside autograd backward passes
        _wgrad16(X, G, part, partb, ks, mode)


def _wgrad16(X, G, part, partb, ks, mode):
    xs = X.double().permute(0, 5, 1, 2, 3, 4)           # [V,16,I,J,K,L]
    gs = G.double().permute(0, 5, 1, 2, 3, 4)
    part.zero_()
    partb.zero_()
    if mode == 2:
        V, _, I, J, K, L = xs.shape
        xx = xs.permute(0, 2, 3, 1, 4, 5).reshape(V * I * J, 16, K, L).requires_grad_(False)
        gg = gs.permute(0, 2, 3, 1, 4, 5).reshape(V * I * J, 16, K, L)
        w = torch.zeros(16, 16, ks, ks, dtype=torch.float64, requires_grad=True)
        (F.conv2d(xx, w, padding=ks // 2) * gg).sum().backward()
        part[0, 0] = w.grad.permute(2, 3, 1, 0).reshape(ks * ks, 16, 16).float()   # [tap, ci, co]
    else:
        w = torch.zeros(16, 16, ks, ks, ks, ks, dtype=torch.float64, requires_grad=True)
        (ref.conv4d(xs, ref.conv4d_weight_from_std(w)) * gs).sum().backward()
        # [co, ci, di, dj, dk, dl] -> [dd = di*ks+dj, tap = dk*ks+dl, ci, co]
        part[0] = w.grad.permute(2, 3, 4, 5, 1, 0).reshape(ks * ks, ks * ks, 16, 16).float()
    partb[0] = gs.sum(dim=(0, 2, 3, 4, 5)).float()


def wgrad16p(X, G, part, partb, ks):
    """Plane-only partials of every (X set, G operand) pair (one of them single)."""
    nx, ng = X.shape[0], G.shape[0]
    part.zero_()
    partb.zero_()
    for i in range(nx):
        for n in range(ng):
            p1 = torch.zeros((2, 1, ks * ks, 16, 16))
            pb = torch.zeros((2, 16))
            wgrad16(X[i], G[n], p1, pb, ks, 2, 2)
            part[0, i * ng + n] = p1[0, 0]
            partb[0, i * ng + n] = pb[0]


def _shift_ij(x, si, sj):
    """out[:, i, j] = x[:, i + si, j + sj] (zero outside), x [V, I, J, ...]."""
    I, J = x.shape[1], x.shape[2]
    out = torch.zeros_like(x)
    ilo, ihi, jlo, jhi = max(0, -si), min(I, I - si), max(0, -sj), min(J, J - sj)
    if ilo < ihi and jlo < jhi:
        out[:, ilo:ihi, jlo:jhi] = x[:, ilo + si:ihi + si, jlo + sj:jhi + sj]
    return out


def ijpack(X, S, ks, sgn):
    x = X.double()
    P = ks // 2
    S.zero_()
    for q in range(ks * ks):
        S[q // 16, ..., q % 16] = _shift_ij(x, sgn * (q // ks - P), sgn * (q % ks - P)).to(S.dtype)


def ijsum(Z, bias, y, ks, relu, sgn):
    P = ks // 2
    acc = torch.zeros(y.shape, dtype=torch.float64)
    for q in range(ks * ks):
        acc += _shift_ij(Z[q].double(), sgn * (q // ks - P), sgn * (q % ks - P))
    if bias is not None:
        acc += float(bias[0])
    y.copy_(torch.relu(acc) if relu else acc)


def combine_fwd(z, y, R, C):
    z = z.reshape(-1)
    Vh = y.numel() // (R * C)
    z1, z2 = z[:Vh * R * C].view(Vh, R, C), z[Vh * R * C:].view(Vh, C, R)
    y.view(Vh, R, C).copy_(z1 + z2.transpose(1, 2))


def combine_bwd(g, z, gz, R, C, gzl=None):
    z = z.reshape(-1)
    Vh = g.numel() // (R * C)
    z1, z2 = z[:Vh * R * C].view(Vh, R, C), z[Vh * R * C:].view(Vh, C, R)
    g3 = g.view(Vh, R, C)
    full = torch.cat(((g3 * (z1 > 0)).reshape(-1), (g3.transpose(1, 2) * (z2 > 0)).reshape(-1)))
    gz.reshape(-1).copy_(full)
    if gzl is not None:
        gzl.reshape(-1).copy_(full - gz.reshape(-1).float())


def _split_into(out_hi, out_lo, y):
    out_hi.copy_(y)
    out_lo.copy_(y - out_hi.double())


def conv16_fwd_x3(X, Xl, Wp2, bias, M, Y, Yl, ks, epi):
    """bf16x3 layer: conv(Xh, Wh) + conv(Xh, Wl) + conv(Xl, Wh) in fp64, then the
    epilogue, written split (hi, lo)."""
    shp = tuple(Y.shape)
    outs = []
    for xx, ww in ((X, Wp2[0]), (X, Wp2[1]), (Xl, Wp2[0])):
        z = torch.empty((16,) + shp[:5], dtype=torch.float32)
        conv16_fwd(xx, ww, None, None, z, ks, 4)
        outs.append(z.double())
    y = (outs[0] + outs[1] + outs[2]).permute(1, 2, 3, 4, 5, 0)
    if epi == 1:
        y = torch.relu(y + bias.double())
    else:
        y = y * (M.double() > 0)
    _split_into(Y, Yl, y)


def conv16_blk_fwd_x3(X, Xl, Wp2, bias, Y, ks, relu):
    acc = 0
    for xx, ww in ((X, Wp2[0]), (X, Wp2[1]), (Xl, Wp2[0])):
        z = torch.empty(Y.shape, dtype=torch.float64)
        conv16_blk_fwd(xx, ww, None, z, ks, 0)
        acc = acc + z
    if bias is not None:
        acc = acc + float(bias.reshape(-1)[0])
    Y.copy_(torch.relu(acc) if relu else acc)


def transpose(x, y):
    y.copy_(x.transpose(1, 2))


class EmuExt:
    """Namespace with the binding names used by ops/neigh_consensus.py and ops/conv4d.py."""
    conv16_fwd = staticmethod(conv16_fwd)
    conv16_blk_fwd = staticmethod(conv16_blk_fwd)
    conv16_fwd_x3 = staticmethod(conv16_fwd_x3)
    conv16_blk_fwd_x3 = staticmethod(conv16_blk_fwd_x3)
    wgrad16 = staticmethod(wgrad16)
    wgrad16p = staticmethod(wgrad16p)
    ijpack = staticmethod(ijpack)
    ijsum = staticmethod(ijsum)
    combine_fwd = staticmethod(combine_fwd)
    combine_bwd = staticmethod(combine_bwd)
    transpose = staticmethod(transpose)
