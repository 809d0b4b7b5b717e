"""CPU emulation of the HIP kernels' fragment layouts and index math.

The MFMA operand maps (cdna_hip_programming.md section 3) are applied to the
packed weights exactly as the kernels read them, and the result is compared
with the PyTorch Conv4d oracle.  This pins the conv16 weight packing, the
data-gradient weight flip and the ij encoding of the 1-channel layers
(forward, data and weight gradients) without a GPU.
"""
import math

import pytest
import torch

from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.packing import pack_w16, transpose_for_dgrad

torch.manual_seed(0)


def _rand_w(cout, cin, ks):
    return torch.randn(cout, cin, ks, ks, ks, ks, dtype=torch.float64)


def _pad_plane(x, i, j, k0, l0, pr, rs, P):
    """Zero-padded [pr, rs, C] window of volume x[I,J,K,L,C] with corner (k0-P, l0-P)."""
    I, J, K, L, C = x.shape
    out = torch.zeros(pr, rs, C, dtype=x.dtype)
    if not (0 <= i < I and 0 <= j < J):
        return out
    for r in range(pr):
        kg = k0 - P + r
        if 0 <= kg < K:
            lo, hi = max(0, l0 - P), min(L, l0 - P + rs)
            out[r, lo - (l0 - P):hi - (l0 - P)] = x[i, j, kg, lo:hi]
    return out


@pytest.mark.parametrize("ks", [3, 5])
def test_pack_w16_roundtrip(ks):
    w = _rand_w(16, 16, ks).float()
    wp = pack_w16(w).float()  # [dd, q, lane, j]
    nt = ks * ks
    rec = torch.zeros(16, 16, ks * ks, nt)
    for q in range(wp.shape[1]):
        for lane in range(64):
            tap = 2 * q + (lane >> 5)
            co = lane & 15
            for j in range(8):
                ci = 8 * ((lane >> 4) & 1) + j
                if tap < nt:
                    rec[co, ci, :, tap] = wp[:, q, lane, j]
                else:
                    assert torch.all(wp[:, q, lane, j] == 0)
    assert torch.equal(rec.reshape(w.shape), w.to(torch.bfloat16).float())


@pytest.mark.parametrize("ks", [3, 5])
def test_dgrad_weights_are_flipped_transpose(ks):
    # dX of a conv == conv of dY with transpose_for_dgrad(W)
    x = torch.randn(1, 3, 4, 4, 5, 5, dtype=torch.float64, requires_grad=True)
    w = _rand_w(2, 3, ks)
    y = ref.conv4d(x, ref.conv4d_weight_from_std(w))
    g = torch.randn_like(y)
    (y * g).sum().backward()
    gx = ref.conv4d(g, ref.conv4d_weight_from_std(transpose_for_dgrad(w)))
    assert torch.allclose(gx, x.grad, atol=1e-9)


def _ijpack(x, ks, sgn):
    """torch emulation of csrc/jshift.hip ijpack: x [V,I,J,K,L] -> [G,V,16,I,J,K,L]."""
    V, I, J, K, L = x.shape
    P = ks // 2
    G = (ks * ks + 15) // 16
    out = torch.zeros(G, V, 16, I, J, K, L, dtype=x.dtype)
    for q in range(ks * ks):
        si, sj = sgn * (q // ks - P), sgn * (q % ks - P)
        ilo, ihi, jlo, jhi = max(0, -si), min(I, I - si), max(0, -sj), min(J, J - sj)
        out[q // 16, :, q % 16, ilo:ihi, jlo:jhi] = x[:, ilo + si:ihi + si, jlo + sj:jhi + sj]
    return out


def _ijsum(z, ks, sgn):
    """emulation of ijsum: z [G,V,16,I,J,K,L] -> [V,I,J,K,L]."""
    G, V, _, I, J, K, L = z.shape
    P = ks // 2
    y = torch.zeros(V, I, J, K, L, dtype=z.dtype)
    for q in range(ks * ks):
        si, sj = sgn * (q // ks - P), sgn * (q % ks - P)
        ilo, ihi, jlo, jhi = max(0, -si), min(I, I - si), max(0, -sj), min(J, J - sj)
        y[:, ilo:ihi, jlo:jhi] += z[q // 16, :, q % 16, ilo + si:ihi + si, jlo + sj:jhi + sj]
    return y


def _plane_conv(x, wp):
    """(dk, dl)-only conv on every (i, j) plane: x [V,16,I,J,K,L], wp [16 out, 16 in, k, k]."""
    V, C, I, J, K, L = x.shape
    ks = wp.shape[-1]
    xx = x.permute(0, 2, 3, 1, 4, 5).reshape(V * I * J, C, K, L)
    y = torch.nn.functional.conv2d(xx, wp, padding=ks // 2)
    return y.reshape(V, I, J, -1, K, L).permute(0, 3, 1, 2, 4, 5)


def _plane_wgrad(x, g, ks):
    """sum over voxels of x[vox + tap][ci] * g[vox][co] -> [tap, ci, co] (wgrad16 plane-only mode)."""
    xa = x.clone().requires_grad_(True)
    w = torch.zeros(16, 16, ks, ks, dtype=x.dtype, requires_grad=True)   # [co, ci, dk, dl]
    (_plane_conv(xa, w) * g).sum().backward()
    return w.grad.permute(2, 3, 1, 0).reshape(ks * ks, 16, 16)


@pytest.mark.parametrize("ks", [1, 3, 5, 7])
def test_ij_encoding_forward_and_grads(ks):
    """Both plane offsets in channels: 1->16 layer == sum_g planeconv(ijpack(x)[g], W_g),
    16->1 layer == ijsum(planeconv(x, W_g)), weight grads via ij_in_grad / ij_out_grad,
    data grads via plane_dgrad_weights + ijpack(-1) / ijsum(-1)."""
    from ncnet_amd.ops.packing import (ij_groups, ij_in_grad, ij_in_weights, ij_out_grad, ij_out_weights,
                                       plane_dgrad_weights)
    torch.manual_seed(4)
    V, I, J, K, L = 2, 5, 6, 5, 4
    G = ij_groups(ks)
    # Cin = 1
    x0 = torch.randn(V, I, J, K, L, dtype=torch.float64)
    w1 = _rand_w(16, 1, ks)
    y_ref = ref.conv4d(x0.unsqueeze(1), ref.conv4d_weight_from_std(w1))
    wi = ij_in_weights(w1)
    xs = _ijpack(x0, ks, 1)
    y_ij = sum(_plane_conv(xs[g], wi[g]) for g in range(G))
    assert torch.allclose(y_ij, y_ref, atol=1e-9)
    g1 = torch.randn_like(y_ref)
    w_a = w1.clone().requires_grad_(True)
    x0a = x0.clone().requires_grad_(True)
    (ref.conv4d(x0a.unsqueeze(1), ref.conv4d_weight_from_std(w_a)) * g1).sum().backward()
    s = torch.stack([_plane_wgrad(xs[g], g1, ks) for g in range(G)])   # [G, tap, c, co]
    assert torch.allclose(ij_in_grad(s, 16), w_a.grad, atol=1e-9)
    wd = plane_dgrad_weights(wi)
    z = torch.stack([_plane_conv(g1, wd[g]) for g in range(G)])
    assert torch.allclose(_ijsum(z, ks, -1), x0a.grad, atol=1e-9)
    # Cout = 1
    x2 = torch.randn(V, 16, I, J, K, L, dtype=torch.float64)
    w3 = _rand_w(1, 16, ks)
    y3_ref = ref.conv4d(x2, ref.conv4d_weight_from_std(w3))[:, 0]
    wo = ij_out_weights(w3)
    z3 = torch.stack([_plane_conv(x2, wo[g]) for g in range(G)])
    assert torch.allclose(_ijsum(z3, ks, 1), y3_ref, atol=1e-9)
    g3 = torch.randn_like(y3_ref)
    assert torch.allclose((_ijsum(z3, ks, 1) * g3).sum(), (z3 * _ijpack(g3, ks, -1)).sum())
    w3_a = w3.clone().requires_grad_(True)
    x2a = x2.clone().requires_grad_(True)
    (ref.conv4d(x2a, ref.conv4d_weight_from_std(w3_a))[:, 0] * g3).sum().backward()
    gs = _ijpack(g3, ks, -1)
    s3 = torch.stack([_plane_wgrad(x2, gs[g], ks) for g in range(G)])  # [G, tap, ci, c]
    assert torch.allclose(ij_out_grad(s3, 16), w3_a.grad, atol=1e-9)
    wd3 = plane_dgrad_weights(wo)
    dx2 = sum(_plane_conv(gs[g], wd3[g]) for g in range(G))
    assert torch.allclose(dx2, x2a.grad, atol=1e-9)
