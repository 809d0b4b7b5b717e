"""CPU emulation of the HIP kernels' fragment layouts and index math.

The MFMA operand maps (cdna_hip_programming.md section 3) are applied to the
packed weights exactly as the kernels read them, and the result is compared
with the PyTorch Conv4d oracle.  This pins the weight packing, the 4x4 shift
grid of the Cout=1 kernel and the staging origins / tap flips of the
1-channel weight-gradient kernel without a GPU.
"""
import math

import pytest
import torch

from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.packing import pack_w16, pack_w1in, pack_w1out, transpose_for_dgrad

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
def test_pack_w1in_roundtrip(ks):
    w = _rand_w(16, 1, ks).float()
    wp = pack_w1in(w).float()
    rec = torch.zeros(16, ks * ks, ks, ks)
    for m in range(wp.shape[1]):
        for lane in range(64):
            dk = 4 * m + (lane >> 4)
            co = lane & 15
            for j in range(8):
                if dk < ks and j < ks:
                    rec[co, :, dk, j] = wp[:, m, lane, j]
                else:
                    assert torch.all(wp[:, m, lane, j] == 0)
    assert torch.equal(rec.reshape(16, 1, ks, ks, ks, ks), w.to(torch.bfloat16).float())


def _emulate_conv1out(x, wp, ks):
    """Kernel algorithm of conv1out_fwd for one volume x [I,J,K,L,16] (K, L <= 25)."""
    I, J, K, L, _ = x.shape
    P, TS = ks // 2, ks + 3
    na, nb = math.ceil(K / 4), math.ceil(L / 4)
    pr, rs = 4 * na + ks - 1, 4 * nb + ks - 1
    y = torch.zeros(I, J, K, L, dtype=torch.float64)
    # W'[dd, tau, s, ci]
    wq = torch.zeros(ks * ks, TS * TS, 16, 16, dtype=torch.float64)
    for p in range(wp.shape[1]):
        for lane in range(64):
            tau = 2 * p + (lane >> 5)
            if tau >= TS * TS:
                continue
            s = lane & 15
            for jj in range(8):
                ci = 8 * ((lane >> 4) & 1) + jj
                wq[:, tau, s, ci] = wp[:, p, lane, jj].double()
    for i in range(I):
        for j in range(J):
            acc = torch.zeros(16, na, nb, dtype=torch.float64)  # [s, ak, al]
            for di in range(ks):
                for dj in range(ks):
                    ii, jj2 = i + di - P, j + dj - P
                    if not (0 <= ii < I and 0 <= jj2 < J):
                        continue
                    plane = _pad_plane(x, ii, jj2, 0, 0, pr, rs, P)  # [pr, rs, 16]
                    dd = di * ks + dj
                    for tau in range(TS * TS):
                        tk, tl = divmod(tau, TS)
                        xs = plane[tk:tk + 4 * na:4, tl:tl + 4 * nb:4]  # [na, nb, ci]
                        acc += torch.einsum("sc,abc->sab", wq[dd, tau], xs)
            for s in range(16):
                sk, sl = divmod(s, 4)
                for ak in range(na):
                    for al in range(nb):
                        k, l = 4 * ak + sk, 4 * al + sl
                        if k < K and l < L:
                            y[i, j, k, l] = acc[s, ak, al]
    return y


@pytest.mark.parametrize("ks,shape", [(3, (3, 4, 6, 7)), (5, (5, 3, 9, 6))])
def test_conv1out_shift_grid(ks, shape):
    I, J, K, L = shape
    x = torch.randn(I, J, K, L, 16, dtype=torch.float64).to(torch.bfloat16).double()
    w = _rand_w(1, 16, ks).to(torch.bfloat16).double()
    wp = pack_w1out(w.float())
    y = _emulate_conv1out(x, wp, ks)
    yr = ref.conv4d(x.permute(4, 0, 1, 2, 3).unsqueeze(0), ref.conv4d_weight_from_std(w))[0, 0]
    assert torch.allclose(y, yr, atol=1e-9, rtol=1e-9)


def _emulate_wgrad1(S16, P1, ks, mode):
    """Kernel algorithm of wgrad1 (one volume; whole plane = one tile).
    S16 [I,J,K,L,16], P1 [I,J,K,L]; returns part [dd, tap, 16]."""
    I, J, K, L, _ = S16.shape
    P = ks // 2
    TK, TL = K, L
    if mode == 0:
        SR, SCV, s_ok, p_ok = TK, TL, 0, -P
    else:
        SR, SCV, s_ok, p_ok = TK + ks - 1, TL + ks - 1, -P, -(ks - 1)
    SC = (SCV + 7) // 8 * 8
    PRR, PWC = SR + ks - 1, SC + ks - 1
    RW = PWC + 8
    out = torch.zeros(ks * ks, ks * ks, 16, dtype=torch.float64)
    for di in range(ks):
        for dj in range(ks):
            dd = di * ks + dj
            for i in range(I):
                for j in range(J):
                    ii, jj = i + di - P, j + dj - P
                    if not (0 <= ii < I and 0 <= jj < J):
                        continue
                    si, sj = (i, j) if mode == 0 else (ii, jj)
                    pi, pj = (ii, jj) if mode == 0 else (i, j)
                    S = torch.zeros(SR + 1, SC, 16, dtype=torch.float64)
                    for r in range(SR):
                        for c in range(SCV):
                            kg, lg = s_ok + r, s_ok + c
                            inbox = (0 <= kg < K and 0 <= lg < L)
                            if inbox:
                                S[r, c] = S16[si, sj, kg, lg]
                    Pr = torch.zeros(PRR + 1, RW, dtype=torch.float64)
                    for r in range(PRR):
                        for c in range(RW):
                            kg, lg = p_ok + r, p_ok + c
                            if mode == 1:
                                ok = 0 <= kg < TK and 0 <= lg < TL
                            else:
                                ok = 0 <= kg < K and 0 <= lg < L
                            if ok:
                                Pr[r, c] = P1[pi, pj, kg, lg]
                    for tap in range(ks * ks):
                        dk, dl = divmod(tap, ks)
                        # sum over S positions (r, c): S[r,c,:] * P[r+dk, c+dl]
                        pv = Pr[dk:dk + SR, dl:dl + SC]
                        out[dd, tap] += torch.einsum("rcx,rc->x", S[:SR], pv)
    return out


@pytest.mark.parametrize("ks", [3, 5])
def test_wgrad1_mode0_layer_in(ks):
    # layer Cin=1 -> Cout=16: dW[co, 0, d] = sum_o G[o, co] X[o + d - P]
    I, J, K, L = 3, 3, 5, 6
    X = torch.randn(I, J, K, L, dtype=torch.float64)
    G = torch.randn(I, J, K, L, 16, dtype=torch.float64)
    part = _emulate_wgrad1(G, X, ks, 0)
    from ncnet_amd.ops.neigh_consensus import _reduce_wgrad1
    dw = _reduce_wgrad1(part.unsqueeze(0), ks, 0, 16)
    w = torch.zeros(16, 1, ks, ks, ks, ks, dtype=torch.float64, requires_grad=True)
    y = ref.conv4d(X.unsqueeze(0).unsqueeze(0), ref.conv4d_weight_from_std(w))
    (y * G.permute(4, 0, 1, 2, 3).unsqueeze(0)).sum().backward()
    assert torch.allclose(dw, w.grad, atol=1e-9)


@pytest.mark.parametrize("ks", [3, 5])
def test_wgrad1_mode1_layer_out(ks):
    # layer Cin=16 -> Cout=1: dW[0, ci, d] = sum_o X[o + d - P, ci] G[o]
    I, J, K, L = 3, 4, 6, 5
    X = torch.randn(I, J, K, L, 16, dtype=torch.float64)
    G = torch.randn(I, J, K, L, dtype=torch.float64)
    part = _emulate_wgrad1(X, G, ks, 1)
    from ncnet_amd.ops.neigh_consensus import _reduce_wgrad1
    dw = _reduce_wgrad1(part.unsqueeze(0), ks, 1, 16)
    w = torch.zeros(1, 16, ks, ks, ks, ks, dtype=torch.float64, requires_grad=True)
    y = ref.conv4d(X.permute(4, 0, 1, 2, 3).unsqueeze(0), ref.conv4d_weight_from_std(w))
    (y[0, 0] * G).sum().backward()
    assert torch.allclose(dw, w.grad, atol=1e-9)


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


def _jpack(x, ks, sgn):
    """torch emulation of csrc/jshift.hip jpack: x [V,I,J,K,L] -> [V,16,I,J,K,L] (channels-first)."""
    V, I, J, K, L = x.shape
    P = ks // 2
    out = torch.zeros(V, 16, I, J, K, L, dtype=x.dtype)
    for c in range(ks):
        s = sgn * (c - P)
        lo, hi = max(0, -s), min(J, J - s)
        out[:, c, :, lo:hi] = x[:, :, lo + s:hi + s]
    return out


def _jsum(z, ks, sgn):
    """emulation of jsum: z [V,16,I,J,K,L] -> [V,I,J,K,L], y[j] = sum_c z[c][j + sgn*(c-P)]."""
    V, _, I, J, K, L = z.shape
    P = ks // 2
    y = torch.zeros(V, I, J, K, L, dtype=z.dtype)
    for c in range(ks):
        s = sgn * (c - P)
        lo, hi = max(0, -s), min(J, J - s)
        y[:, :, lo:hi] += z[:, c, :, lo + s:hi + s]
    return y


@pytest.mark.parametrize("ks", [3, 5])
def test_jchannel_encoding_forward_and_grads(ks):
    """1->16 layer == conv16_{dj=P}(jpack(x)) and 16->1 layer == jsum(conv16_{dj=P}(x)),
    including the weight-gradient maps jc_in_grad / jc_out_grad."""
    from ncnet_amd.ops.packing import jc_in_grad, jc_in_weights, jc_out_grad, jc_out_weights
    torch.manual_seed(3)
    V, I, J, K, L = 2, 4, 6, 5, 5
    P = ks // 2
    # Cin = 1
    x0 = torch.randn(V, I, J, K, L, dtype=torch.float64)
    w1 = _rand_w(16, 1, ks)
    y_ref = ref.conv4d(x0.unsqueeze(1), ref.conv4d_weight_from_std(w1))
    wj = jc_in_weights(w1)
    assert torch.count_nonzero(wj[:, :, :, [d for d in range(ks) if d != P]]) == 0
    xs = _jpack(x0, ks, 1)
    y_j = ref.conv4d(xs, ref.conv4d_weight_from_std(wj))
    assert torch.allclose(y_j, y_ref, atol=1e-9)
    g = torch.randn_like(y_ref)
    w_a = w1.clone().requires_grad_(True)
    (ref.conv4d(x0.unsqueeze(1), ref.conv4d_weight_from_std(w_a)) * g).sum().backward()
    wj_a = wj.clone().requires_grad_(True)
    (ref.conv4d(xs, ref.conv4d_weight_from_std(wj_a)) * g).sum().backward()
    s5 = wj_a.grad[:, :, :, P]  # [co, ci, di, dk, dl]
    assert torch.allclose(jc_in_grad(s5, 16), w_a.grad, atol=1e-9)
    # Cout = 1
    x2 = torch.randn(V, 16, I, J, K, L, dtype=torch.float64)
    w3 = _rand_w(1, 16, ks)
    y3_ref = ref.conv4d(x2, ref.conv4d_weight_from_std(w3))[:, 0]
    wz = jc_out_weights(w3)
    z = ref.conv4d(x2, ref.conv4d_weight_from_std(wz))
    assert torch.allclose(_jsum(z, ks, 1), y3_ref, atol=1e-9)
    g3 = torch.randn_like(y3_ref)
    # adjoint: jsum(+1)^T == jpack(-1)
    assert torch.allclose((_jsum(z, ks, 1) * g3).sum(), (z * _jpack(g3, ks, -1)).sum())
    w3_a = w3.clone().requires_grad_(True)
    (ref.conv4d(x2, ref.conv4d_weight_from_std(w3_a))[:, 0] * g3).sum().backward()
    wz_a = wz.clone().requires_grad_(True)
    (ref.conv4d(x2, ref.conv4d_weight_from_std(wz_a)) * _jpack(g3, ks, -1)).sum().backward()
    assert torch.allclose(jc_out_grad(wz_a.grad[:, :, :, P], 16), w3_a.grad, atol=1e-9)
    # data gradient of the Cin=1 layer: jsum(-1) of the dj=P transposed conv
    x0a = x0.clone().requires_grad_(True)
    (ref.conv4d(x0a.unsqueeze(1), ref.conv4d_weight_from_std(w1)) * g).sum().backward()
    dxs = ref.conv4d(g, ref.conv4d_weight_from_std(transpose_for_dgrad(wj)))
    assert torch.allclose(_jsum(dxs, ks, -1), x0a.grad, atol=1e-9)


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


@pytest.mark.parametrize("ks", [3, 5])
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
