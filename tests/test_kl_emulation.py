"""CPU emulation of the kl kernels (csrc/conv4d_kl.hip).

The kernels' index math -- output tiles, halo-extended plane staging, the
per-tap LDS offset table of conv1to16_kl, the plane pairing / zero-weight
padding and the in-LDS combo shift-sum of conv16to1_kl -- is replayed in
float64 from the packed weights exactly as the kernels read them, and
compared with the PyTorch Conv4d oracle (ops/reference.py).
"""
import pytest
import torch

from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.packing import kl_dgrad_in_weights, pack_kl_in, pack_kl_out

torch.manual_seed(0)


def _tiles(K, L, TK, TL):
    for k0 in range(0, K, TK):
        for l0 in range(0, L, TL):
            yield k0, l0


def _emulate_conv1to16_kl(x, wp, ks, TK, TL):
    """x [V,I,J,K,L]; wp [NS, 64, 8] -> y [V,I,J,K,L,16] (no epilogue)."""
    V, I, J, K, L = x.shape
    P, NC = ks // 2, ks * ks
    NS = wp.shape[0]
    PR, RW = TK + ks - 1, TL + ks - 1
    psz = PR * RW
    wfull = torch.zeros(NS * 32, 16, dtype=torch.float64)       # [tap, co]
    for s in range(NS):
        for lane in range(64):
            for j in range(8):
                wfull[32 * s + 8 * (lane >> 4) + j, lane & 15] = float(wp[s, lane, j])
    tab = torch.zeros(NS * 32, dtype=torch.long)
    for kk in range(NC * NC):
        p, q = divmod(kk, NC)
        dk, dl = divmod(q, ks)
        tab[kk] = p * psz + dk * RW + dl
    y = torch.zeros(V, I, J, K, L, 16, dtype=torch.float64)
    for v in range(V):
        for i in range(I):
            for j in range(J):
                for k0, l0 in _tiles(K, L, TK, TL):
                    xt = torch.zeros(NC, PR, RW, dtype=torch.float64)
                    for p in range(NC):
                        di, dj = divmod(p, ks)
                        ii, jj = i + di - P, j + dj - P
                        if not (0 <= ii < I and 0 <= jj < J):
                            continue
                        for r in range(PR):
                            kg = k0 - P + r
                            if not 0 <= kg < K:
                                continue
                            for c in range(RW):
                                lg = l0 - P + c
                                if 0 <= lg < L:
                                    xt[p, r, c] = x[v, ii, jj, kg, lg]
                    flat = xt.reshape(-1)
                    kk, ll = torch.meshgrid(torch.arange(TK), torch.arange(TL), indexing="ij")
                    vb = (kk * RW + ll).reshape(-1)
                    im = flat[vb[:, None] + tab[None, :]]                 # [voxels, taps]
                    out = (im @ wfull).reshape(TK, TL, 16)
                    ke, le = min(K, k0 + TK), min(L, l0 + TL)
                    y[v, i, j, k0:ke, l0:le] = out[:ke - k0, :le - l0]
    return y


def _emulate_conv16to1_kl(h, wl, ks, TK, TL):
    """h [V,I,J,K,L,16]; wl [k*k+1, NCT, 16, 16] -> y [V,I,J,K,L] (no bias / ReLU)."""
    V, I, J, K, L, _ = h.shape
    P, NT = ks // 2, ks * ks
    NCT = wl.shape[1]
    PR, RW = TK + ks - 1, TL + ks - 1
    ne = PR * RW
    wlf = wl.double()
    y = torch.zeros(V, I, J, K, L, dtype=torch.float64)
    for v in range(V):
        for i in range(I):
            for j in range(J):
                di_lo, di_hi = max(0, P - i), min(ks, I + P - i)
                dj_lo, dj_hi = max(0, P - j), min(ks, J + P - j)
                ndj = dj_hi - dj_lo
                planes = [(di_lo + s // ndj) * ks + dj_lo + s % ndj for s in range((di_hi - di_lo) * ndj)]
                for k0, l0 in _tiles(K, L, TK, TL):
                    z = torch.zeros(NCT * 16, ne, dtype=torch.float64)
                    for q in range((len(planes) + 1) // 2):
                        pair = [planes[2 * q], planes[2 * q + 1] if 2 * q + 1 < len(planes) else planes[2 * q]]
                        wsel = [pair[0], pair[1] if 2 * q + 1 < len(planes) else NT]
                        for half in range(2):
                            p = pair[half]
                            di, dj = divmod(p, ks)
                            buf = torch.zeros(PR, RW, 16, dtype=torch.float64)
                            for r in range(PR):
                                kg = k0 - P + r
                                if 0 <= kg < K:
                                    for c in range(RW):
                                        lg = l0 - P + c
                                        if 0 <= lg < L:
                                            buf[r, c] = h[v, i + di - P, j + dj - P, kg, lg]
                            a = wlf[wsel[half]].reshape(NCT * 16, 16)           # [combo, ch]
                            z += a @ buf.reshape(ne, 16).T
                    zz = z[:NT].reshape(NT, PR, RW)
                    for kk in range(min(TK, K - k0)):
                        for ll in range(min(TL, L - l0)):
                            s = 0.0
                            for dk in range(ks):
                                for dl in range(ks):
                                    s += zz[dk * ks + dl, kk + dk, ll + dl]
                            y[v, i, j, k0 + kk, l0 + ll] = s
    return y


def _oracle(x_ncijkl, w_std):
    return ref.conv4d(x_ncijkl, ref.conv4d_weight_from_std(w_std))


@pytest.mark.parametrize("ks,shape,tk,tl", [(3, (1, 4, 3, 5, 7), 3, 4), (5, (1, 3, 4, 6, 5), 6, 5),
                                             (5, (2, 5, 5, 5, 5), 2, 3)])
def test_conv1to16_kl_forward(ks, shape, tk, tl):
    x = torch.randn(*shape, dtype=torch.float64)
    w = torch.randn(16, 1, ks, ks, ks, ks, dtype=torch.float64)
    wp = pack_kl_in(w).double()
    got = _emulate_conv1to16_kl(x, wp, ks, tk, tl)
    want = _oracle(x.unsqueeze(1), w.to(torch.bfloat16).double()).permute(0, 2, 3, 4, 5, 1)
    assert torch.allclose(got, want, atol=1e-9), (got - want).abs().max()


@pytest.mark.parametrize("ks,cout", [(3, 16), (5, 10)])
def test_conv1to16_kl_dgrad_of_cout1_layer(ks, cout):
    """The Cout=1 layer's data gradient is conv1to16_kl with flipped, transposed taps."""
    cin = cout
    shape = (1, 3, 4, 5, 4)
    w = torch.randn(1, cin, ks, ks, ks, ks, dtype=torch.float64)
    x = torch.randn(1, cin, *shape[1:], dtype=torch.float64, requires_grad=True)
    g = torch.randn(1, 1, *shape[1:], dtype=torch.float64)
    wb = w.to(torch.bfloat16).double()
    y = _oracle(x, wb)
    (gx,) = torch.autograd.grad(y, x, g)
    wp = pack_kl_in(kl_dgrad_in_weights(w)).double()
    got = _emulate_conv1to16_kl(g[:, 0], wp, ks, 5, 4)[..., :cin]
    assert torch.allclose(got, gx.permute(0, 2, 3, 4, 5, 1), atol=1e-9)


@pytest.mark.parametrize("ks,shape,tk,tl,cin", [(3, (1, 4, 3, 5, 7), 3, 4, 16), (5, (1, 4, 3, 6, 5), 4, 5, 16),
                                                 (5, (1, 5, 5, 5, 5), 5, 5, 12), (3, (2, 2, 2, 3, 3), 3, 3, 16)])
def test_conv16to1_kl_forward(ks, shape, tk, tl, cin):
    h = torch.randn(*shape, 16, dtype=torch.float64)
    h[..., cin:] = 0
    w = torch.randn(1, cin, ks, ks, ks, ks, dtype=torch.float64)
    wl = pack_kl_out(w)
    assert tuple(wl.shape) == (ks * ks + 1, (ks * ks + 15) // 16, 16, 16)
    assert torch.all(wl[-1] == 0)
    got = _emulate_conv16to1_kl(h, wl, ks, tk, tl)
    want = _oracle(h[..., :cin].permute(0, 5, 1, 2, 3, 4), w.to(torch.bfloat16).double())[:, 0]
    assert torch.allclose(got, want, atol=1e-9), (got - want).abs().max()


# ---------------------------------------------------------------------------
# nc_fused_k3 (csrc/nc_fused.hip): the streaming schedule, replayed.

def _emulate_nc_fused(x0, w1, b1, w2, b2, TK, TL, R, IR):
    """Plane-by-plane replay of the fused kernel: S tile gather -> layer-1
    plane conv (ij weights) on the tile + 1 halo, zero outside the volume ->
    layer-2 combo conv -> 3-row ring at (ih - di2 + 1, j'' - dj2 + 1) -> flush."""
    import torch.nn.functional as F
    from ncnet_amd.ops.packing import ij_in_weights, ij_out_weights
    V, I, J, K, L = x0.shape
    W1 = ij_in_weights(w1)[0].double()           # [16 co, 16 c=(di1,dj1), 3, 3]
    W2 = ij_out_weights(w2)[0].double()          # [16 q=(di2,dj2), 16 ci, 3, 3]
    b1p = torch.zeros(16, dtype=torch.float64)
    b1p[:b1.numel()] = b1.double()
    y = torch.full((V, I, J, K, L), float("nan"), dtype=torch.float64)
    for v in range(V):
        for i0 in range(0, I, IR):
            i1 = min(I, i0 + IR)
            for j0 in range(0, J, R):
                Rv = min(R, J - j0)
                for k0 in range(0, K, TK):
                    for l0 in range(0, L, TL):
                        ring = torch.zeros(3, R, TK, TL, dtype=torch.float64)
                        ih_lo, ih_hi = max(0, i0 - 1), min(I, i1 + 1)
                        jh_lo, jh_hi = max(0, j0 - 1), min(J, j0 + Rv + 1)

                        def flush(io):
                            for p in range(Rv):
                                for kk in range(TK):
                                    for ll in range(TL):
                                        if k0 + kk < K and l0 + ll < L:
                                            y[v, io, j0 + p, k0 + kk, l0 + ll] = max(ring[io % 3, p, kk, ll] + float(b2), 0.0)
                            ring[io % 3] = 0

                        for ih in range(ih_lo, ih_hi):
                            for jh in range(jh_lo, jh_hi):
                                S = torch.zeros(16, TK + 4, TL + 4, dtype=torch.float64)
                                for c in range(9):
                                    ii, jj = ih + c // 3 - 1, jh + c % 3 - 1
                                    if not (0 <= ii < I and 0 <= jj < J):
                                        continue
                                    for r in range(TK + 4):
                                        for cc in range(TL + 4):
                                            kg, lg = k0 - 2 + r, l0 - 2 + cc
                                            if 0 <= kg < K and 0 <= lg < L:
                                                S[c, r, cc] = x0[v, ii, jj, kg, lg]
                                h = torch.relu(F.conv2d(S[None], W1)[0] + b1p.view(16, 1, 1))   # [16, TK+2, TL+2]
                                kin = torch.tensor([0 <= k0 - 1 + r < K for r in range(TK + 2)])
                                lin = torch.tensor([0 <= l0 - 1 + c < L for c in range(TL + 2)])
                                h = h * (kin[:, None] & lin[None, :])
                                z = F.conv2d(h[None], W2)[0]                                   # [16 combos, TK, TL]
                                for c in range(9):
                                    io, p = ih - c // 3 + 1, jh - c % 3 + 1 - j0
                                    if i0 <= io < i1 and 0 <= p < Rv:
                                        ring[io % 3, p] += z[c]
                            if i0 <= ih - 1 < i1:
                                flush(ih - 1)
                        for io in range(max(i0, ih_hi - 1), i1):
                            flush(io)
    return y


@pytest.mark.parametrize("shape,tiles", [((1, 5, 6, 7, 8), (3, 4, 2, 2)), ((2, 4, 3, 5, 5), (5, 5, 3, 4)),
                                         ((1, 6, 5, 4, 9), (2, 3, 4, 3))])
def test_nc_fused_schedule(shape, tiles):
    from ncnet_amd.ops.neigh_consensus import fused_tiles
    torch.manual_seed(3)
    x0 = torch.rand(*shape, dtype=torch.float64)
    w1 = torch.randn(16, 1, 3, 3, 3, 3, dtype=torch.float64) * 0.3
    b1 = torch.randn(16, dtype=torch.float64) * 0.1
    w2 = torch.randn(1, 16, 3, 3, 3, 3, dtype=torch.float64) * 0.3
    b2 = torch.tensor([0.05], dtype=torch.float64)
    got = _emulate_nc_fused(x0, w1, b1, w2, b2, *tiles)
    h = torch.relu(_oracle(x0.unsqueeze(1), w1) + b1.view(1, 16, 1, 1, 1, 1))
    want = torch.relu(_oracle(h, w2) + b2)[:, 0]
    assert not torch.isnan(got).any(), "every output voxel must be flushed exactly once"
    assert torch.allclose(got, want, atol=1e-9), (got - want).abs().max()
    tk, tl, R, IR = fused_tiles(*shape)
    assert (tk + 2) * (tl + 2) <= 512 and tk * tl <= 384 and (tk + 4) * (tl + 4) <= 512 and R >= 1 and IR >= 1
