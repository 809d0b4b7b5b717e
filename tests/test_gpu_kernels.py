"""HIP kernel numerics vs the PyTorch fp32/fp64 oracles (run on an MI355X).

Inputs are rounded to bf16 first and the oracle runs in fp64 on those values,
so the remaining differences are fp32 accumulation order and the bf16 rounding
of stored activations.
"""
import os
import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(x):
    return x.to(torch.bfloat16).double()


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def rel_l2(a, b):
    """||a - b|| / ||b||: robust to the few ReLU-mask flips that bf16 activations
    cause in a multi-layer composite (a flip moves one element by its full value)."""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def test_extension_loaded():
    assert _ext.available(), "HIP extension must load on the GPU box"
    import ncnet_amd._C as C  # noqa: F401


@pytest.mark.parametrize("ks,shape", [(5, (2, 25, 25, 25, 25)), (3, (1, 7, 9, 11, 13)), (3, (1, 3, 2, 30, 27)),
                                      (5, (1, 6, 5, 26, 29)), (5, (1, 4, 12, 9, 7)), (7, (1, 9, 8, 25, 25)),
                                      (7, (1, 4, 5, 30, 28)), (1, (2, 5, 6, 25, 25))])
def test_conv16_fwd(ks, shape):
    """conv16 forward: v3 (X reused over 5 output j-planes, KS 3/5) and v2
    (one plane per workgroup, KS 1/7), multi-tile K, L."""
    from ncnet_amd.ops.packing import pack_w16
    torch.manual_seed(0)
    V, I, J, K, L = shape
    x = torch.rand(V, 16, I, J, K, L, device=DEV)
    w = torch.randn(16, 16, ks, ks, ks, ks, device=DEV) * 0.05
    b = torch.randn(16, device=DEV) * 0.1
    xcl = x.permute(0, 2, 3, 4, 5, 1).contiguous().to(torch.bfloat16)
    y = torch.empty_like(xcl)
    _ext.ext().conv16_fwd(xcl, pack_w16(w), b, None, y, ks, 1)
    yr = torch.relu(ref.conv4d(bf(x), ref.conv4d_weight_from_std(bf(w)), b.double()))
    assert relerr(y.permute(0, 5, 1, 2, 3, 4), yr) < 1e-2


@pytest.mark.parametrize("epi", [1, 2])
@pytest.mark.parametrize("shape", [(2, 25, 25, 25, 25), (1, 6, 7, 26, 29), (1, 4, 6, 50, 37), (1, 3, 11, 25, 25)])
def test_conv16v4_matches_v3_bitwise(epi, shape, monkeypatch, tune):
    """conv16v4 (compile-time 25 x 25 tile: pipelined fragments, triple-buffered
    planes with counted vmcnt, buffer-resource DMA that writes the halo zeros)
    accumulates every output in conv16v3's order: bit-identical outputs for the
    forward (bias + ReLU) and data-gradient (ReLU-mask) epilogues, including
    partial (k, l) tiles and j-blocks, and against the fp64 oracle."""
    from ncnet_amd.ops.packing import pack_w16
    torch.manual_seed(1)
    V, I, J, K, L = shape
    x = torch.rand(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    m = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    w_std = torch.randn(16, 16, 5, 5, 5, 5, device=DEV) * 0.05
    w = pack_w16(w_std)
    b = torch.randn(16, device=DEV) * 0.1
    outs = []
    for v3 in ("0", "1"):
        tune("conv_v3", v3)
        y = torch.full_like(x, float("nan"))
        _ext.ext().conv16_fwd(x, w, b if epi == 1 else None, m if epi == 2 else None, y, 5, epi)
        outs.append(y)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])
    # and v4 itself against the fp64 oracle on the same bf16 operands: bias +
    # ReLU (forward) or the ReLU mask of the previous activation (the data
    # gradient's EPI_MASK epilogue)
    z = ref.conv4d(x.double().permute(0, 5, 1, 2, 3, 4), ref.conv4d_weight_from_std(bf(w_std)), None)
    if epi == 1:
        want = torch.relu(z + b.double().view(1, 16, 1, 1, 1, 1))
    else:
        want = z * (m.double().permute(0, 5, 1, 2, 3, 4) > 0)
    got = outs[0].permute(0, 5, 1, 2, 3, 4)
    # the only difference is the final bf16 rounding of the stored output (2^-9)
    assert relerr(got, want) < 4e-3, relerr(got, want)


@pytest.mark.parametrize("ks,T", [(5, 20), (5, 15), (3, 25), (3, 20), (3, 15), (5, 30), (3, 30)])
@pytest.mark.parametrize("epi", [1, 2])
def test_conv16v4_other_planes(ks, T, epi, tune):
    """conv16v4 at the other compile-time training planes (--image_size 320 /
    240 / 480 -- the 30 x 30 plane as two 30 x 15 tiles -- and k = 3):
    bit-identical to the general conv16v3 at the same tiles and within the
    final bf16 rounding of the fp64 oracle."""
    from ncnet_amd.ops.packing import pack_w16
    torch.manual_seed(2)
    V, I, J = 2, 7, 11
    x = torch.rand(V, I, J, T, T, 16, device=DEV).to(torch.bfloat16)
    m = torch.randn(V, I, J, T, T, 16, device=DEV).to(torch.bfloat16)
    w_std = torch.randn(16, 16, ks, ks, ks, ks, device=DEV) * 0.05
    w = pack_w16(w_std)
    b = torch.randn(16, device=DEV) * 0.1
    outs = []
    for v3 in ("0", "1"):
        tune("conv_v3", v3)
        y = torch.full_like(x, float("nan"))
        _ext.ext().conv16_fwd(x, w, b if epi == 1 else None, m if epi == 2 else None, y, ks, epi)
        outs.append(y)
    assert torch.isfinite(outs[0].float()).all()
    z = ref.conv4d(x.double().permute(0, 5, 1, 2, 3, 4), ref.conv4d_weight_from_std(bf(w_std)), None)
    want = torch.relu(z + b.double().view(1, 16, 1, 1, 1, 1)) if epi == 1 else z * (m.double().permute(0, 5, 1, 2, 3, 4) > 0)
    e4, e3 = relerr(outs[0].permute(0, 5, 1, 2, 3, 4), want), relerr(outs[1].permute(0, 5, 1, 2, 3, 4), want)
    print(f"conv16v4 k{ks} {T}x{T}: v4 {e4:.2e} v3 {e3:.2e} bitwise {torch.equal(outs[0], outs[1])}")
    assert e4 < 4e-3 and e3 < 4e-3, (e4, e3)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("ks,T", [(5, 20), (5, 15), (3, 25), (3, 20), (3, 15), (5, 30), (3, 30)])
def test_wgrad16v4_other_planes(ks, T, tune):
    """wgrad16v4 at the other compile-time planes vs the general wgrad16v3 and
    the fp64 weight gradient.  (5, 30): 34-voxel X rows, two DMA instructions
    per row -- wgrad16v3 cannot stage them, so only the fp64 check applies."""
    from ncnet_amd.ops.neigh_consensus import wgrad16_partials, _reduce_wgrad16
    torch.manual_seed(9)
    V, I, J = 2, 6, 9
    x = torch.randn(V, I, J, T, T, 16, device=DEV).to(torch.bfloat16)
    g = torch.randn(V, I, J, T, T, 16, device=DEV).to(torch.bfloat16)
    res = []
    for v3 in (("0",) if T + ks - 1 > 32 else ("0", "1")):
        tune("wgrad_v3", v3)
        s, sb = wgrad16_partials(_ext.ext(), x, g, ks, False)
        res.append((_reduce_wgrad16(s, ks, 16, 16), sb))
    w = torch.zeros(ks, 16, 16, ks, ks, ks, device=DEV, dtype=torch.float64, requires_grad=True)
    y = ref.conv4d(x.double().permute(0, 5, 1, 2, 3, 4), w, None)
    (y * g.double().permute(0, 5, 1, 2, 3, 4)).sum().backward()
    want = ref.conv4d_weight_to_std(w.grad)
    for dw, db in res:
        assert relerr(dw, want) < 1e-4, relerr(dw, want)
        assert relerr(db, g.double().sum(dim=(0, 1, 2, 3, 4))) < 1e-4


@pytest.mark.parametrize("ks,shape,cin,relu", [(5, (4, 25, 25, 25, 25), 16, 1), (5, (1, 6, 5, 26, 29), 16, 0),
                                               (3, (2, 7, 9, 11, 13), 10, 1), (3, (1, 3, 2, 30, 27), 16, 1),
                                               (7, (1, 9, 8, 25, 25), 16, 1), (1, (2, 5, 6, 25, 25), 16, 0),
                                               (5, (1, 13, 11, 9, 7), 16, 1)])
def test_conv16_blk_fwd(ks, shape, cin, relu):
    """Cout=1 conv in output-plane-block mode (4x4 output planes per
    workgroup = the 16 MFMA rows, partial blocks at the I/J edges, multi-tile
    K, L) vs the fp64 Conv4d oracle."""
    from ncnet_amd.ops.packing import blk_out_weights, pack_w16_planes
    torch.manual_seed(1)
    V, I, J, K, L = shape
    x = torch.rand(V, cin, I, J, K, L, device=DEV)
    w = torch.randn(1, cin, ks, ks, ks, ks, device=DEV) * 0.05
    b = torch.randn(1, device=DEV) * 0.1 - (0.3 if relu else 0.0)
    xcl = torch.zeros(V, I, J, K, L, 16, device=DEV, dtype=torch.bfloat16)
    xcl[..., :cin] = x.permute(0, 2, 3, 4, 5, 1).to(torch.bfloat16)
    y = torch.full((V, I, J, K, L), float("nan"), device=DEV)
    _ext.ext().conv16_blk_fwd(xcl, pack_w16_planes(blk_out_weights(w)), b, y, ks, relu)
    yr = ref.conv4d(bf(x), ref.conv4d_weight_from_std(bf(w)), b.double())[:, 0]
    if relu:
        yr = torch.relu(yr)
    assert torch.isfinite(y).all()
    assert relerr(y, yr) < 1e-4


@pytest.mark.parametrize("shape,cin,relu", [((3, 25, 25, 25, 25), 16, 1), ((2, 25, 25, 25, 25), 16, 0),
                                          ((1, 7, 10, 25, 25), 16, 1), ((1, 1, 1, 25, 25), 16, 0),
                                          ((2, 4, 3, 25, 25), 10, 1)])
def test_cout1_taps_fwd(shape, cin, relu):
    """Cout=1 conv with the 25 in-plane taps on the MFMA rows (csrc/cout1.hip:
    2 x 2 output-plane items, odd I / J edges, the in-plane shift-sum through
    LDS) vs the fp64 Conv4d oracle on the same bf16 operands, and bit for bit
    across two launches; a one-tap weight perturbation must be detected."""
    from ncnet_amd.ops.packing import cout1_taps_weights
    torch.manual_seed(3)
    ks = 5
    V, I, J, K, L = shape
    x = torch.rand(V, cin, I, J, K, L, device=DEV)
    w = torch.randn(1, cin, ks, ks, ks, ks, device=DEV) * 0.05
    b = torch.randn(1, device=DEV) * 0.1 - (0.3 if relu else 0.0)
    xcl = torch.zeros(V, I, J, K, L, 16, device=DEV, dtype=torch.bfloat16)
    xcl[..., :cin] = x.permute(0, 2, 3, 4, 5, 1).to(torch.bfloat16)
    wt = cout1_taps_weights(w).to(torch.bfloat16)
    y = torch.full((V, I, J, K, L), float("nan"), device=DEV)
    assert _ext.ext().cout1_taps_fwd(xcl, wt, b, y, ks, relu)
    yr = ref.conv4d(bf(x), ref.conv4d_weight_from_std(bf(w)), b.double())[:, 0]
    if relu:
        yr = torch.relu(yr)
    assert torch.isfinite(y).all()
    assert relerr(y, yr) < 1e-4, relerr(y, yr)
    y2 = torch.full_like(y, float("nan"))
    _ext.ext().cout1_taps_fwd(xcl, wt, b, y2, ks, relu)
    assert torch.equal(y, y2)
    # mutation: one tap of the centre (di, dj) plane (used by every output) off by a visible amount
    wm = w.clone()
    wm[0, 3, 2, 2, 4, 0] += 0.5
    ym = torch.empty_like(y)
    _ext.ext().cout1_taps_fwd(xcl, cout1_taps_weights(wm).to(torch.bfloat16), b, ym, ks, relu)
    assert relerr(ym, yr) > 1e-3
    # other planes: the launcher declines (the caller keeps the block kernel)
    xs = torch.zeros(1, 3, 3, 20, 20, 16, device=DEV, dtype=torch.bfloat16)
    assert not _ext.ext().cout1_taps_fwd(xs, wt, b, torch.empty(1, 3, 3, 20, 20, device=DEV), ks, relu)


@pytest.mark.parametrize("ks,shape,nx,ng", [(5, (2, 25, 25, 25, 25), 1, 2), (5, (2, 25, 25, 25, 25), 2, 1),
                                            (3, (2, 7, 9, 11, 13), 1, 1), (7, (1, 9, 8, 25, 25), 1, 2),
                                            (1, (2, 5, 6, 20, 25), 2, 1)])
def test_wgrad16p(ks, shape, nx, ng):
    """Double-buffered plane-only weight gradient (both ij groups per launch)
    vs the fp64 plane-conv definition: dW[tap][ci][co] = sum X[vox + tap] G[vox]."""
    import torch.nn.functional as F
    torch.manual_seed(2)
    V, I, J, K, L = shape
    x = (torch.rand((nx,) + shape + (16,), device=DEV) - 0.3).to(torch.bfloat16)
    g = torch.randn((ng,) + shape + (16,), device=DEV).to(torch.bfloat16)
    part = torch.full((64, nx * ng, ks * ks, 16, 16), float("nan"), device=DEV)
    partb = torch.full((64, nx * ng, 16), float("nan"), device=DEV)
    _ext.ext().wgrad16p(x, g, part, partb, ks)
    s, sb = part.sum(0), partb.sum(0)
    for a in range(nx):
        for n in range(ng):
            xx = x[a].double().reshape(V * I * J, K, L, 16).permute(0, 3, 1, 2)
            gg = g[n].double().reshape(V * I * J, K, L, 16).permute(0, 3, 1, 2)
            P = ks // 2
            xp = F.pad(xx, (P, P, P, P))
            want = torch.stack([torch.einsum("nckl,nokl->co", xp[:, :, dk:dk + K, dl:dl + L], gg)
                                for dk in range(ks) for dl in range(ks)])   # [tap, ci, co]
            assert relerr(s[a * ng + n], want) < 1e-4
            assert relerr(sb[a * ng + n], gg.sum(dim=(0, 2, 3))) < 1e-4


@pytest.mark.parametrize("cin,cout,ks", [(16, 16, 5), (1, 16, 5), (16, 1, 5), (16, 16, 3), (1, 16, 3), (16, 1, 3),
                                         (10, 10, 3), (32, 16, 3), (1, 40, 3), (24, 1, 5), (16, 16, 7), (1, 16, 7),
                                         (16, 16, 1), (1, 1, 3), (20, 33, 3)])
def test_conv4d_autograd(cin, cout, ks):
    """The Conv4d module on the HIP path for any channel counts / kernel sizes 1-7."""
    from ncnet_amd.ops.conv4d import conv4d
    torch.manual_seed(3)
    shape = (2, cin, 9, 8, 11, 10)
    x = torch.rand(shape, device=DEV).to(torch.bfloat16).float().requires_grad_(True)
    w = (torch.randn(ks, cout, cin, ks, ks, ks, device=DEV) * 0.05).to(torch.bfloat16).float().requires_grad_(True)
    b = (torch.randn(cout, device=DEV) * 0.1).requires_grad_(True)
    before = _ext.DISPATCH["conv4d_hip"]
    y = conv4d(x, w, b, permute_filters=False)
    assert _ext.DISPATCH["conv4d_hip"] == before + 1
    g = torch.randn_like(y).to(torch.bfloat16).float()
    (y * g).sum().backward()
    xr, wr, br = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = ref.conv4d(xr, wr, br)
    (yr * g.double()).sum().backward()
    assert relerr(y, yr) < 1e-2
    assert relerr(x.grad, xr.grad) < 2e-2
    assert relerr(w.grad, wr.grad) < 2e-2
    assert relerr(b.grad, br.grad) < 1e-3


def test_conv4d_even_kernel_raises_without_opt_in(runtime):
    """No silent fallback: k = 4 has no HIP kernel, so the GPU op raises unless
    NCNET_ALLOW_TORCH_FALLBACK=1 opts into the PyTorch reference."""
    from ncnet_amd.ops.conv4d import conv4d
    x = torch.rand(1, 16, 4, 4, 4, 4, device=DEV)
    w = torch.randn(4, 16, 16, 4, 4, 4, device=DEV) * 0.05
    runtime(allow_torch_fallback=False)
    with pytest.raises(NotImplementedError):
        conv4d(x, w, None, permute_filters=False)


@pytest.mark.parametrize("ks,ch,shape", [((5, 5, 5), (16, 16, 1), (2, 1, 12, 12, 12, 12)),
                                         ((3, 3), (16, 1), (2, 1, 10, 11, 10, 11)),
                                         ((3, 3), (16, 1), (1, 1, 8, 10, 9, 7)),
                                         ((3, 3, 3), (10, 10, 1), (2, 1, 9, 9, 9, 9)),
                                         ((5, 5), (32, 1), (1, 1, 10, 9, 10, 9)),
                                         ((7, 3), (16, 1), (1, 1, 9, 10, 9, 10))])
def test_neigh_consensus_autograd(ks, ch, shape):
    from ncnet_amd.ops.neigh_consensus import neigh_consensus
    torch.manual_seed(4)
    x = torch.rand(shape, device=DEV).to(torch.bfloat16).float().requires_grad_(True)
    ws, bs = [], []
    cin = 1
    for k, c in zip(ks, ch):
        ws.append((torch.randn(k, c, cin, k, k, k, device=DEV) * 0.1).to(torch.bfloat16).float().requires_grad_(True))
        # positive biases keep most units active: a last layer with ~2% active units makes its bias
        # gradient a sum of ~100 terms where one bf16-induced ReLU flip moves it by 10-30%
        bs.append((0.5 + torch.rand(c, device=DEV) * 0.1).requires_grad_(True))
        cin = c
    before = _ext.DISPATCH["nc_bf16"]
    y = neigh_consensus(x, ws, bs, list(ch), symmetric=True)
    assert _ext.DISPATCH["nc_bf16"] == before + 1     # the HIP autograd stack, not a fallback
    g = torch.randn_like(y)
    (y * g).sum().backward()
    xr = x.detach().double().requires_grad_(True)
    wr = [w.detach().double().requires_grad_(True) for w in ws]
    br = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wr, br, symmetric=True)
    (yr * g.double()).sum().backward()
    errs = {"y": rel_l2(y, yr), "gx": rel_l2(x.grad, xr.grad)}
    for li, (a, r) in enumerate(zip(ws, wr)):
        errs[f"gw{li}"] = rel_l2(a.grad, r.grad)
    for li, (a, r) in enumerate(zip(bs, br)):
        errs[f"gb{li}"] = rel_l2(a.grad, r.grad)
    # vs the UNquantized fp64 oracle the bf16 activations/gradients cost a few %;
    # tests/test_gpu_nc_stages.py checks every stage tightly vs a quantized oracle.
    assert errs["y"] < 1e-2 and max(errs.values()) < 0.1, errs


@pytest.mark.parametrize("shape", [(3, 1, 25, 25, 25, 25), (2, 1, 7, 9, 11, 5), (2, 1, 8, 10, 16, 20)])
def test_mutual_matching(shape):
    from ncnet_amd.ops.mutual import mutual_matching
    torch.manual_seed(5)
    c = torch.rand(shape, device=DEV, requires_grad=True)
    y = mutual_matching(c)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    cr = c.detach().double().requires_grad_(True)
    yr = ref.mutual_matching(cr)
    (yr * g.double()).sum().backward()
    assert relerr(y, yr) < 1e-5
    assert relerr(c.grad, cr.grad) < 1e-4


def test_l2norm_and_correlation():
    from ncnet_amd.ops.correlation import correlation, l2norm_pack
    torch.manual_seed(6)
    f = torch.relu(torch.randn(4, 1024, 25, 25, device=DEV)).contiguous(memory_format=torch.channels_last)
    p = l2norm_pack(f)
    pr = ref.feature_l2norm(f.double()).reshape(4, 1024, 625).transpose(1, 2)
    assert relerr(p, pr) < 1e-2
    amap = torch.tensor([0, 1, 1, 0], device=DEV, dtype=torch.int32)
    bmap = torch.tensor([2, 3, 2, 3], device=DEV, dtype=torch.int32)
    c = correlation(p, p, amap, bmap)
    cr = torch.bmm(p.double()[amap.long()], p.double()[bmap.long()].transpose(1, 2))
    assert relerr(c, cr) < 1e-3


def test_correlation_odd_sizes_and_grad():
    from ncnet_amd.ops.correlation import correlation
    torch.manual_seed(7)
    a = torch.randn(2, 77, 40, device=DEV).to(torch.bfloat16).float().requires_grad_(True)
    b = torch.randn(2, 131, 40, device=DEV).to(torch.bfloat16).float().requires_grad_(True)
    c = correlation(a, b)
    g = torch.randn_like(c)
    (c * g).sum().backward()
    ar, br = a.detach().double().requires_grad_(True), b.detach().double().requires_grad_(True)
    cr = torch.bmm(ar, br.transpose(1, 2))
    (cr * g.double()).sum().backward()
    assert relerr(c, cr) < 1e-3
    assert relerr(a.grad, ar.grad) < 1e-3 and relerr(b.grad, br.grad) < 1e-3


@pytest.mark.parametrize("norm", ["softmax", "l1", None])
def test_weak_loss_scores(norm):
    """All three weak-loss normalisations (train.py:111-116) on the HIP stats +
    closed-form backward kernels, vs autograd of the fp64 oracle."""
    from ncnet_amd.ops.loss import weak_loss_from_corr
    torch.manual_seed(8)
    x = (torch.rand(4, 1, 6, 7, 6, 7, device=DEV) * 3).requires_grad_(True)
    loss = weak_loss_from_corr(x, 2, norm)
    loss.backward()
    xr = x.detach().double().requires_grad_(True)
    lr = ref.match_score(xr[2:], norm) - ref.match_score(xr[:2], norm)
    lr.backward()
    assert abs(float(loss) - float(lr)) < 1e-5 * max(1.0, abs(float(lr)))
    assert relerr(x.grad, xr.grad) < 1e-4


def test_maxpool4d_and_fused_pool():
    from ncnet_amd.ops.correlation import correlation, correlation_pool2, maxpool4d
    torch.manual_seed(9)
    v = torch.rand(2, 1, 6, 8, 4, 10, device=DEV)
    val, off = maxpool4d(v, 2)
    vr, offr = ref.maxpool4d(v.cpu(), 2)
    assert torch.equal(val.cpu(), vr)
    for a, b in zip(off, offr):
        assert torch.equal(a.cpu().long(), b.long())
    fa = torch.randn(2, 6 * 8, 64, device=DEV).to(torch.bfloat16).float()
    fb = torch.randn(2, 4 * 10, 64, device=DEV).to(torch.bfloat16).float()
    pv, po = correlation_pool2(fa, fb, 6, 8, 4, 10)
    full = correlation(fa, fb).view(2, 1, 6, 8, 4, 10)
    rv, ro = ref.maxpool4d(full.cpu(), 2)
    assert relerr(pv, rv) < 1e-5
    agree = sum(int(torch.equal(a.cpu().long(), b.long())) for a, b in zip(po, ro))
    assert agree == 4


def test_correlation_v2_large_grids():
    """The LDS-DMA-ring correlation GEMM (corr_gemm_v2, chosen for >= 512
    workgroups: InLoc volumes) with ragged M / N edges and batch maps: plain
    store vs an fp64 GEMM, fused 2x2x2x2 max-pool vs pooling the full volume."""
    from ncnet_amd.ops.correlation import correlation, correlation_pool2, maxpool4d
    torch.manual_seed(10)
    hA, wA, hB, wB = 66, 70, 58, 74
    fa = torch.nn.functional.normalize(torch.randn(2, hA * wA, 1024, device=DEV), dim=-1).to(torch.bfloat16).float()
    fb = torch.nn.functional.normalize(torch.randn(2, hB * wB, 1024, device=DEV), dim=-1).to(torch.bfloat16).float()
    amap = torch.tensor([1, 0], device=DEV, dtype=torch.int32)
    bmap = torch.tensor([0, 0], device=DEV, dtype=torch.int32)
    c = correlation(fa, fb, amap, bmap)
    cr = torch.bmm(fa.double()[amap.long()], fb.double()[bmap.long()].transpose(1, 2))
    assert relerr(c, cr) < 1e-5
    pv, po = correlation_pool2(fa, fb, hA, wA, hB, wB)
    full = correlation(fa, fb).view(2, 1, hA, wA, hB, wB)
    rv, ro = maxpool4d(full, 2)
    assert relerr(pv, rv) < 1e-6
    for a, b in zip(po, ro):
        assert (a.long() == b.long()).float().mean() > 0.999
    # the MX-fp8 v2 kernel (corr_gemm_f8v2): same grids on e4m3 operands vs fp64 on the same values
    from ncnet_amd.ops.correlation import FP8, FP8_FEAT_SCALE
    qa, qb = (fa * FP8_FEAT_SCALE).to(FP8), (fb * FP8_FEAT_SCALE).to(FP8)
    c8 = correlation(qa, qb, amap, bmap)
    cr8 = torch.bmm(qa.double()[amap.long()], qb.double()[bmap.long()].transpose(1, 2)) / FP8_FEAT_SCALE ** 2
    assert relerr(c8, cr8) < 1e-4   # fp32 accumulation order (near-zero random correlations)
    pv8, po8 = correlation_pool2(qa, qb, hA, wA, hB, wB)
    full8 = correlation(qa, qb).view(2, 1, hA, wA, hB, wB)
    rv8, ro8 = maxpool4d(full8, 2)
    assert relerr(pv8, rv8) < 1e-6
    for a, b in zip(po8, ro8):
        assert (a.long() == b.long()).float().mean() > 0.999


@pytest.mark.parametrize("shape,ng", [((2, 6, 5, 25, 25), 7), ((3, 25, 25, 25, 25), 102), ((1, 4, 7, 25, 25), 1),
                                      ((2, 9, 3, 25, 25), 40)])
def test_wgrad16v4_matches_v3(shape, ng, monkeypatch, tune):
    """wgrad16v4 (compile-time 25 x 25 plane: X and G DMA'd two steps ahead with
    counted vmcnt, buffer-resource zero halo, per-tap-group specialised body)
    walks the same columns, steps and chunks as wgrad16v3, so every partial
    accumulates in the same order: identical partials (and the fp64 oracle
    bound), incl. group counts that leave some workgroups without columns and
    dj offsets whose columns are skipped."""
    C = _ext.ext()
    torch.manual_seed(12)
    x = torch.rand(shape + (16,), device=DEV).to(torch.bfloat16)
    g = torch.randn(shape + (16,), device=DEV).to(torch.bfloat16)
    outs = []
    for v3 in ("0", "1"):
        tune("wgrad_v3", v3)
        part = torch.full((2 * ng, 25, 25, 16, 16), float("nan"), device=DEV)
        partb = torch.full((2 * ng, 16), float("nan"), device=DEV)
        C.wgrad16(x, g, part, partb, 5, 0, 3)
        outs.append((part, partb))
    assert torch.isfinite(outs[0][0]).all() and torch.isfinite(outs[0][1]).all()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("variant", [2, 3])
@pytest.mark.parametrize("ks,shape", [(5, (2, 6, 5, 25, 25)), (5, (1, 5, 4, 30, 27)), (3, (1, 4, 5, 9, 33)),
                                      (5, (1, 2, 3, 7, 6)), (7, (1, 3, 4, 25, 25)), (1, (1, 3, 4, 25, 26))])
def test_wgrad16_kernel(variant, ks, shape):
    """Weight / bias gradient of a 16->16 Conv4d straight from the wgrad16
    kernels (v3 sliding ring for KS 3/5 when the row fits, v2 per plane
    offset; multi-tile K, L exercise the per-item halo), full and plane-only
    modes, vs autograd of the fp64 oracle."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    C = _ext.ext()
    torch.manual_seed(11)
    V, I, J, K, L = shape
    if variant == 3 and not nc.wgrad_v3_ok(shape, ks):
        pytest.skip("wgrad16v3 needs KS 3/5 and L + KS - 1 <= 32")
    x = torch.rand(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    g = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    xr = x.double().permute(0, 5, 1, 2, 3, 4)
    wr = torch.zeros(ks, 16, 16, ks, ks, ks, device=DEV, dtype=torch.float64, requires_grad=True)
    yr = ref.conv4d(xr, wr, None)
    (yr * g.double().permute(0, 5, 1, 2, 3, 4)).sum().backward()
    dstd = ref.conv4d_weight_to_std(wr.grad)           # [co, ci, di, dj, dk, dl]
    if variant == 3:
        ng = nc.wgrad_v3_groups(shape, ks)
    else:
        ng = nc.wgrad_groups(ks, nc._nitems(shape))
    part = torch.empty((2 * ng, ks * ks, ks * ks, 16, 16), device=DEV)
    partb = torch.empty((2 * ng, 16), device=DEV)
    C.wgrad16(x, g, part, partb, ks, 0, variant)
    dw = nc._reduce_wgrad16(part.sum(0), ks, 16, 16)
    assert relerr(dw, dstd) < 1e-3
    assert relerr(partb.sum(0), g.double().sum(dim=(0, 1, 2, 3, 4))) < 1e-3
    sp, sbp = nc.wgrad16_partials(C, x, g, ks, True)     # plane-only: the (P, P) offset
    P = ks // 2
    assert relerr(sp[0].permute(2, 1, 0).reshape(16, 16, ks, ks), dstd[:, :, P, P]) < 1e-3
    assert relerr(sbp, partb.sum(0)) < 1e-5


@pytest.mark.parametrize("flags", ["0", "1"])
def test_wgrad16v3_priority_flag(flags, monkeypatch, tune):
    """wgrad16v3 with the waves-4..7 s_setprio tuning bit: same sums as the oracle."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    tune("wgrad_flags", flags)
    torch.manual_seed(12)
    V, I, J, K, L, ks = 2, 6, 5, 25, 25, 5
    x = torch.rand(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    g = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    wr = torch.zeros(ks, 16, 16, ks, ks, ks, device=DEV, dtype=torch.float64, requires_grad=True)
    (ref.conv4d(x.double().permute(0, 5, 1, 2, 3, 4), wr, None) * g.double().permute(0, 5, 1, 2, 3, 4)).sum().backward()
    s, sb = nc.wgrad16_partials(_ext.ext(), x, g, ks, False)
    assert relerr(nc._reduce_wgrad16(s, ks, 16, 16), ref.conv4d_weight_to_std(wr.grad)) < 1e-3
    assert relerr(sb, g.double().sum(dim=(0, 1, 2, 3, 4))) < 1e-3


@pytest.mark.parametrize("ks,sgn,shape,dtype", [(5, 1, (2, 6, 7, 25, 25), torch.bfloat16),
                                                (5, -1, (1, 5, 4, 9, 11), torch.float32),
                                                (3, 1, (1, 4, 5, 30, 26), torch.bfloat16),
                                                (3, -1, (2, 3, 3, 7, 5), torch.bfloat16),
                                                (5, 1, (1, 3, 4, 40, 30), torch.bfloat16),
                                                (7, 1, (1, 8, 9, 6, 7), torch.bfloat16),
                                                (1, -1, (1, 3, 4, 6, 7), torch.float32)])
def test_ijpack_kernel(ks, sgn, shape, dtype):
    """ijpack vs the torch emulation of the ij encoding:
    S[g][v,i,j,k,l,c] = X[v, i+sgn*(di-P), j+sgn*(dj-P), k, l], q = 16g + c."""
    from tests.test_kernel_emulation import _ijpack
    torch.manual_seed(13)
    x = torch.randn(shape, device=DEV).to(dtype)
    G = (ks * ks + 15) // 16
    s = torch.full((G,) + shape + (16,), float("nan"), device=DEV, dtype=torch.bfloat16)
    _ext.ext().ijpack(x, s, ks, sgn)
    want = _ijpack(x.float().cpu(), ks, sgn).permute(0, 1, 3, 4, 5, 6, 2).to(torch.bfloat16)
    assert torch.equal(s.cpu(), want)


def test_bias_act_kernel():
    C = _ext.ext()
    torch.manual_seed(5)
    y = torch.randn(2, 64, 9, 7, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, device=DEV)
    ref_ = torch.relu(y.float() + b.view(1, -1, 1, 1))
    C.bias_act_(y, b, 1)
    assert relerr(y, ref_) < 1e-2
    z = torch.randn(33, 128, device=DEV).to(torch.bfloat16)
    refz = z.float() + b.repeat(2)
    C.bias_act_(z, b.repeat(2).contiguous(), 0)
    assert relerr(z, refz) < 1e-2


def test_frozen_trunk_plan_gpu():
    """bf16 GEMM/epilogue execution plan of the frozen ResNet trunk vs the fp32 eager trunk."""
    from ncnet_amd.models.backbones import FrozenResNetPlan, fold_frozen_bn, resnet_trunk
    torch.manual_seed(0)
    t = resnet_trunk("resnet101", "layer3").eval()
    for m in t.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
    t = t.to(DEV)
    x = torch.randn(2, 3, 96, 128, device=DEV)
    with torch.no_grad():
        r = t(x)
        p = FrozenResNetPlan(fold_frozen_bn(t), torch.bfloat16)(x)
    assert p.shape == r.shape
    assert rel_l2(p.float(), r) < 3e-2


def test_frozen_trunk_plan_stem_chunks(monkeypatch):
    """The stem of a batch larger than STEM_CHUNK runs chunk by chunk (each
    chunk's fused bias / ReLU / max-pool writes its slice of one output):
    same features as the unchunked stem, to bf16 rounding."""
    from ncnet_amd.models import backbones as bb
    torch.manual_seed(0)
    t = bb.resnet_trunk("resnet101", "layer3").eval().to(DEV)
    x = torch.randn(5, 3, 96, 128, device=DEV)
    plan = bb.FrozenResNetPlan(bb.fold_frozen_bn(t), torch.bfloat16)
    plan.use_graphs = False
    with torch.no_grad():
        whole = plan(x)
        monkeypatch.setattr(bb, "STEM_CHUNK", 2)
        chunked = plan(x)
    assert chunked.shape == whole.shape
    assert rel_l2(chunked.float(), whole.float()) < 1e-2


def test_fp8_l2norm_and_correlation():
    """fp8 (OCP e4m3) operands: pack kernel vs torch's e4m3 cast, MX-fp8 MFMA
    GEMM (plain and fused 2x2x2x2 pool) vs fp64 math on the same fp8 values.
    Rows are long enough (K = 1024 = 8 MFMA k-blocks) that a wrong lane->k map
    in the K=128 fragments cannot cancel out."""
    from ncnet_amd.ops.correlation import (FP8, FP8_FEAT_SCALE, correlation, correlation_pool2, l2norm_pack_fp8)
    torch.manual_seed(7)
    f = torch.randn(2, 1024, 12, 10, device=DEV).contiguous(memory_format=torch.channels_last)
    y = l2norm_pack_fp8(f)
    assert y.dtype == FP8 and y.shape == (2, 120, 1024)
    yr = (ref.feature_l2norm(f.double()).reshape(2, 1024, 120).transpose(1, 2) * FP8_FEAT_SCALE).float().to(FP8)
    mism = (y.view(torch.uint8) != yr.view(torch.uint8)).float().mean().item()
    assert mism < 1e-3, mism
    fa, fb = y, y.flip(0).contiguous()
    c = correlation(fa, fb)
    cr = torch.bmm(fa.double(), fb.double().transpose(1, 2)) / FP8_FEAT_SCALE ** 2
    assert relerr(c, cr) < 1e-4   # fp32 accumulation order only
    # asymmetric: A rows vs B rows of different images and sizes
    g = torch.randn(1, 1024, 8, 6, device=DEV).contiguous(memory_format=torch.channels_last)
    yb = l2norm_pack_fp8(g)
    c2 = correlation(y[:1], yb)
    cr2 = torch.bmm(y[:1].double(), yb.double().transpose(1, 2)) / FP8_FEAT_SCALE ** 2
    assert relerr(c2, cr2) < 1e-4
    val, (di, dj, dk, dl) = correlation_pool2(fa, fb, 12, 10, 12, 10)
    full = cr.view(2, 1, 12, 10, 12, 10).float()
    vr, *offs = ref.maxpool4d(full, 2)
    assert relerr(val, vr) < 1e-4


def test_immatchnet_fp8_correlation_path():
    """corr_dtype='fp8' inference volumes vs the bf16 path (same weights)."""
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(use_cuda=True, ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1],
                   relocalization_k_size=2).to(DEV).eval()
    batch = {"source_image": torch.randn(1, 3, 256, 320, device=DEV),
             "target_image": torch.randn(1, 3, 256, 320, device=DEV)}
    with torch.inference_mode():
        c16, d16 = m(batch)
        m.corr_dtype = "fp8"
        c8, d8 = m(batch)
    assert c8.shape == c16.shape
    assert rel_l2(c8, c16) < 0.1


@pytest.mark.parametrize("ks,shape", [(5, (2, 25, 25, 25, 25)), (3, (1, 7, 9, 30, 27))])
def test_conv16_fp8_kernel(ks, shape):
    """fp8 (OCP e4m3) inference conv16 vs fp64 math on the same fp8 values:
    bias+ReLU -> fp8 output and planar fp32 output, plain and group-plane mode."""
    from ncnet_amd.ops.packing import pack_w16, pack_w16_planes
    C = _ext.ext()
    F8 = torch.float8_e4m3fn
    torch.manual_seed(21)
    V, I, J, K, L = shape
    x = (torch.rand(V, I, J, K, L, 16, device=DEV) * 2).to(F8)
    w = (torch.randn(16, 16, ks, ks, ks, ks, device=DEV) * 0.05).to(torch.bfloat16).float()
    wsc = 64.0
    wq = (pack_w16(w).float() * wsc).to(F8)
    wr = (w * wsc).to(F8).double() / wsc          # the exact fp8 weight values used
    b = torch.randn(16, device=DEV) * 0.1
    xr = x.double().permute(0, 5, 1, 2, 3, 4)
    yr = ref.conv4d(xr, ref.conv4d_weight_from_std(wr), b.double())
    y = torch.empty((V, I, J, K, L, 16), dtype=F8, device=DEV)
    C.conv16f8_fwd(x, wq, b, y, ks, 1, 1.0 / wsc)
    y_ref = torch.relu(yr).permute(0, 2, 3, 4, 5, 1)
    assert rel_l2(y.float(), y_ref) < 0.04          # e4m3 output rounding (3 mantissa bits)
    # planar fp32, group-plane mode with 2 groups at the (i, j) plane
    wp = (torch.randn(2, 16, 16, ks, ks, device=DEV) * 0.05).to(torch.bfloat16).float()
    wpq = (pack_w16_planes(wp).float() * wsc).to(F8)
    wpr = (wp * wsc).to(F8).double() / wsc
    x2 = (torch.rand(2, V, I, J, K, L, 16, device=DEV) * 2).to(F8)
    z = torch.empty((16, V, I, J, K, L), dtype=torch.float32, device=DEV)
    C.conv16f8_fwd(x2, wpq, None, z, ks, 4, 1.0 / wsc)
    xx = x2.double().permute(0, 1, 2, 3, 6, 4, 5).reshape(2, V * I * J, 16, K, L)
    zr = sum(torch.nn.functional.conv2d(xx[g], wpr[g], padding=ks // 2) for g in range(2))
    zr = zr.reshape(V, I, J, 16, K, L).permute(3, 0, 1, 2, 4, 5)
    assert relerr(z, zr) < 1e-4


def test_immatchnet_fp8_nc_path(runtime):
    """corr_dtype='fp8' with config nc_fp8 (NCNET_NC_FP8=1): fp8 correlation and
    the e4m3 fused NC kernel (nc_fused_k3_f8) for this symmetric (3,3)/(16,1)
    stack, vs the bf16 path; the fp8 Conv4d NC kernels (the nc_fp8 path of
    the other stacks) on the same NC input; without nc_fp8 the fused bf16
    kernel.  The dispatch counters prove which NC implementation ran."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    runtime(nc_fp8=True)
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(use_cuda=True, ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1],
                   relocalization_k_size=2).to(DEV).eval()
    for p in m.NeighConsensus.parameters():   # positive biases: a populated ReLU pattern
        if p.dim() == 1:
            p.data.uniform_(0.05, 0.2)
    batch = {"source_image": torch.randn(1, 3, 256, 320, device=DEV),
             "target_image": torch.randn(1, 3, 256, 320, device=DEV)}
    with torch.inference_mode():
        n_fused, n_f8 = _ext.DISPATCH["nc_fused_k3"], _ext.DISPATCH["nc_fused_k3_f8"]
        c16, _ = m(batch)
        assert _ext.DISPATCH["nc_fused_k3"] == n_fused + 1          # bf16: the fused InLoc kernel
        m.corr_dtype = "fp8"
        c8, _ = m(batch)
        assert _ext.DISPATCH["nc_fused_k3_f8"] == n_f8 + 1          # fp8: the e4m3 fused kernel
        # the fp8 Conv4d stack on a MutualMatching-like input vs the fused fp8 kernel and fp32
        layers = m.NeighConsensus.conv_layers()
        ws, bs = [l.weight_ref() for l in layers], [l.bias for l in layers]
        x = torch.rand(1, 1, 8, 10, 8, 10, device=DEV) ** 3
        n_fp8 = _ext.DISPATCH["nc_fp8"]
        y_conv = nc.neigh_consensus(x, ws, bs, m.NeighConsensus.channels, symmetric=False, fp8=True)
        assert _ext.DISPATCH["nc_fp8"] == n_fp8 + 1
        y_fused = nc.neigh_consensus(x, ws, bs, m.NeighConsensus.channels, symmetric=True, fp8=True)
        y32 = ref.neigh_consensus(x.double(), [w.double() for w in ws], [b.double() for b in bs], symmetric=True)
        y32n = ref.neigh_consensus(x.double(), [w.double() for w in ws], [b.double() for b in bs], symmetric=False)
    assert rel_l2(y_conv, y32n) < 0.15 and rel_l2(y_fused, y32) < 0.05
    assert c8.shape == c16.shape
    assert rel_l2(c8, c16) < 0.15
    runtime(nc_fp8=False)
    with torch.inference_mode():
        n_fused = _ext.DISPATCH["nc_fused_k3"]
        c8f, _ = m(batch)                                         # default fp8 mode: fp8 correlation + fused NC
        assert _ext.DISPATCH["nc_fused_k3"] == n_fused + 1
    assert rel_l2(c8f, c16) < 0.15


def test_nc_forward_deterministic_and_fully_written():
    """Two NC forwards are bitwise equal (no atomics / races) and every output
    voxel is written: the output buffers of the conv kernels are NaN-poisoned
    before launch."""
    from ncnet_amd.ops.neigh_consensus import neigh_consensus
    from ncnet_amd.ops.packing import pack_w16
    torch.manual_seed(13)
    ws = [torch.randn(5, 16, 1, 5, 5, 5, device=DEV) * 0.05, torch.randn(5, 16, 16, 5, 5, 5, device=DEV) * 0.05,
          torch.randn(5, 1, 16, 5, 5, 5, device=DEV) * 0.05]
    bs = [torch.rand(16, device=DEV) * 0.1, torch.rand(16, device=DEV) * 0.1, torch.rand(1, device=DEV) * 0.1]
    x = torch.rand(2, 1, 9, 11, 9, 11, device=DEV)
    with torch.no_grad():
        y1 = neigh_consensus(x, ws, bs, [16, 16, 1])
        y2 = neigh_consensus(x, ws, bs, [16, 16, 1])
    assert torch.equal(y1, y2)
    assert torch.isfinite(y1).all()
    C = _ext.ext()
    xs = torch.rand(2, 9, 11, 30, 27, 16, device=DEV).to(torch.bfloat16)
    w = pack_w16(torch.randn(16, 16, 5, 5, 5, 5, device=DEV) * 0.05)
    y = torch.full_like(xs, float("nan"))
    C.conv16_fwd(xs, w, torch.zeros(16, device=DEV), None, y, 5, 1)
    assert torch.isfinite(y.float()).all()
    z = torch.full((16, 2, 9, 11, 30, 27), float("nan"), device=DEV)
    C.conv16_fwd(xs, w, None, None, z, 5, 4)
    assert torch.isfinite(z).all()


@pytest.mark.parametrize("cin,cout,k,stride,pad,res,relu,shape", [
    (64, 64, 3, 1, 1, False, True, (2, 19, 23)), (128, 256, 1, 1, 0, True, True, (2, 19, 23)),
    (256, 128, 3, 2, 1, False, True, (2, 19, 23)), (64, 256, 1, 2, 0, False, False, (2, 19, 23)),
    (128, 192, 3, 1, 1, True, False, (2, 19, 23)),
    # large enough for the 128-row tiles (>= 512 workgroups)
    (64, 128, 3, 1, 1, True, True, (4, 129, 127)), (64, 64, 1, 1, 0, False, True, (4, 129, 127)),
    # >= 384 tiles of 256 rows: the 8-wave 256 x 128 variant (3x3 / 1x1 + residual / stride 2)
    (64, 128, 3, 1, 1, True, True, (4, 160, 208)), (256, 1024, 1, 1, 0, True, True, (8, 60, 60)),
    (128, 128, 3, 2, 1, False, True, (16, 101, 99))])
def test_conv2d_nhwc_kernel(cin, cout, k, stride, pad, res, relu, shape):
    """NHWC implicit-GEMM conv (+bias, +residual, ReLU) vs F.conv2d in fp64 on bf16 inputs
    (both the 64- and 128-row tile variants)."""
    C = _ext.ext()
    torch.manual_seed(17)
    cl = torch.channels_last
    x = torch.randn(shape[0], cin, shape[1], shape[2], device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=DEV) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(cout, device=DEV)
    yr = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, pad)
    r = None
    if res:
        r = torch.randn(yr.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
        yr = yr + r.double()
    if relu:
        yr = torch.relu(yr)
    y = torch.empty(yr.shape, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=cl)
    C.conv2d_nhwc(x, w, b, r, y, stride, pad, 1 if relu else 0)
    assert relerr(y, yr) < 1e-2


@pytest.mark.parametrize("cin,cout,k,stride,pad,res,relu,shape", [
    (256, 256, 3, 1, 1, False, True, (5, 25, 25)),     # layer-3 3x3 (M = 3125: a partial last 256-row tile)
    (1024, 256, 1, 1, 0, True, True, (3, 25, 25)),     # 1x1 with a residual
    (256, 512, 3, 2, 1, False, False, (2, 30, 31)),    # two 256-column tiles, stride 2, no ReLU
    (64, 256, 1, 1, 0, False, True, (2, 20, 20))])     # Cin 64: two k-steps per tap
def test_conv2d_nhwc_256x256_tile(cin, cout, k, stride, pad, res, relu, shape, tune):
    """The 256 x 256 DMA-ring tile of the Cout = 256 trunk convs (conv2d_nhwc_v2
    <256, 256>, forced by conv2d_variant 4) vs F.conv2d in fp64 on bf16 inputs."""
    tune("conv2d_variant", 4)
    C = _ext.ext()
    torch.manual_seed(23)
    cl = torch.channels_last
    x = torch.randn(shape[0], cin, shape[1], shape[2], device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=DEV) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(cout, device=DEV)
    yr = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, pad)
    r = None
    if res:
        r = torch.randn(yr.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
        yr = yr + r.double()
    if relu:
        yr = torch.relu(yr)
    y = torch.full(yr.shape, float("nan"), dtype=torch.bfloat16, device=DEV).contiguous(memory_format=cl)
    C.conv2d_nhwc(x, w, b, r, y, stride, pad, 1 if relu else 0)
    assert torch.isfinite(y).all()
    assert relerr(y, yr) < 1e-2


@pytest.mark.parametrize("cin,cout,k,stride,pad,res,relu,shape,dt", [
    (256, 256, 3, 1, 1, False, True, (4, 25, 25), torch.bfloat16),     # layer-3 3x3 at the training size
    (1024, 256, 1, 1, 0, False, True, (3, 25, 25), torch.bfloat16),    # layer-3 reduce 1x1
    (256, 1024, 1, 1, 0, True, True, (2, 25, 25), torch.bfloat16),     # layer-3 expand 1x1 + residual
    (256, 256, 3, 2, 1, False, True, (2, 50, 50), torch.bfloat16),     # stride-2 3x3
    (512, 1024, 1, 2, 0, False, False, (2, 50, 50), torch.bfloat16),   # stride-2 downsample
    (128, 128, 3, 1, 1, True, True, (3, 23, 19), torch.bfloat16),      # Cout 128: the 128-column tile
    (256, 256, 3, 1, 1, True, True, (3, 25, 25), torch.float16)])     # IEEE half operands
def test_conv2d_nhwc_v3(cin, cout, k, stride, pad, res, relu, shape, dt, tune):
    """conv2d_nhwc_v3 (one round of chip-sized workgroups: 16 TM x 64 TN tiles,
    8 waves as 2 K-groups x 4 N-groups, LDS-DMA ring, K-group sum in the
    epilogue) vs F.conv2d in fp64 on 16-bit inputs: ragged M, stride 2, residual."""
    C = _ext.ext()
    tune("conv2d_variant", "3")
    torch.manual_seed(18)
    cl = torch.channels_last
    x = torch.randn(shape[0], cin, shape[1], shape[2], device=DEV).to(dt).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=DEV) * 0.05).to(dt).contiguous(memory_format=cl)
    b = torch.randn(cout, device=DEV)
    yr = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, pad)
    r = None
    if res:
        r = torch.randn(yr.shape, device=DEV).to(dt).contiguous(memory_format=cl)
        yr = yr + r.double()
    if relu:
        yr = torch.relu(yr)
    y = torch.full(yr.shape, float("nan"), dtype=dt, device=DEV).contiguous(memory_format=cl)
    C.conv2d_nhwc(x, w, b, r, y, stride, pad, 1 if relu else 0)
    assert torch.isfinite(y.float()).all()
    assert relerr(y, yr) < 1e-2, relerr(y, yr)


@pytest.mark.parametrize("ks,shape", [(5, (2, 6, 7, 25, 25)), (3, (1, 4, 9, 30, 27)), (5, (1, 3, 12, 9, 7))])
def test_group_plane_conv_multitile_bitwise(ks, shape, monkeypatch, tune):
    """The multi-tile group-plane conv16v2 (NCNET_GP_TPW consecutive j-tiles per
    workgroup, one plane stream) does the same MFMAs in the same order as one
    tile per workgroup: outputs are bitwise equal for the bias+ReLU, ReLU-mask
    and planar-fp32 epilogues, including a ragged last j-block; and the bias+ReLU
    output matches the fp64 oracle of the 1 -> 16 layer."""
    from ncnet_amd.ops.packing import ij_groups, ij_in_weights, pack_w16_planes
    torch.manual_seed(14)
    C = _ext.ext()
    V, I, J, K, L = shape
    G = ij_groups(ks)
    x0 = torch.rand(shape, device=DEV).to(torch.bfloat16)
    xs = torch.empty((G,) + shape + (16,), device=DEV, dtype=torch.bfloat16)
    C.ijpack(x0, xs, ks, 1)
    w = torch.randn(16, 1, ks, ks, ks, ks, device=DEV) * 0.1
    b = torch.randn(16, device=DEV) * 0.1
    wp = pack_w16_planes(ij_in_weights(w))
    m = (torch.rand(shape + (16,), device=DEV) > 0.5).to(torch.bfloat16)
    outs = {}
    for tpw in ("1", "5", "3"):
        tune("gp_tpw", tpw)
        y1 = torch.full(shape + (16,), float("nan"), device=DEV, dtype=torch.bfloat16)
        C.conv16_fwd(xs, wp, b, None, y1, ks, 1)
        y2 = torch.full(shape + (16,), float("nan"), device=DEV, dtype=torch.bfloat16)
        C.conv16_fwd(xs, wp, None, m, y2, ks, 2)
        z = torch.full((16,) + shape, float("nan"), device=DEV)
        C.conv16_fwd(xs, wp, None, None, z, ks, 4)
        outs[tpw] = (y1, y2, z)
    for tpw in ("5", "3"):
        for a, r in zip(outs[tpw], outs["1"]):
            assert not torch.isnan(a).any() and torch.equal(a, r)
    yr = torch.relu(ref.conv4d(bf(x0.float()).unsqueeze(1), ref.conv4d_weight_from_std(bf(w)), b.double()))
    assert relerr(outs["5"][0].permute(0, 5, 1, 2, 3, 4), yr) < 1e-2



def test_nontemporal_epilogue_stores_bitwise(monkeypatch, tune):
    """NCNET_NT_STORE=1 (streaming epilogue stores) writes the same bytes as the
    default stores for the v3 16->16 conv, the ReLU-mask data gradient and the
    planar fp32 epilogue (ij-encoded Cout=1 partials)."""
    from ncnet_amd.ops.packing import ij_out_weights, pack_w16, pack_w16_planes
    torch.manual_seed(16)
    C = _ext.ext()
    shape = (2, 6, 7, 25, 25)
    x = torch.rand(shape + (16,), device=DEV).to(torch.bfloat16)
    w = pack_w16(torch.randn(16, 16, 5, 5, 5, 5, device=DEV) * 0.05)
    wz = pack_w16_planes(ij_out_weights(torch.randn(1, 16, 5, 5, 5, 5, device=DEV) * 0.05))[:1]
    b = torch.randn(16, device=DEV) * 0.1
    outs = {}
    for nt in ("0", "1"):
        tune("nt_store", nt)
        y = torch.full_like(x, float("nan"))
        C.conv16_fwd(x, w, b, None, y, 5, 1)
        yd = torch.full_like(x, float("nan"))
        C.conv16_fwd(x, w, None, x, yd, 5, 2)
        z = torch.full((16,) + shape, float("nan"), device=DEV)
        C.conv16_fwd(x.unsqueeze(0), wz, None, None, z, 5, 4)
        outs[nt] = (y, yd, z)
    for a, r in zip(outs["1"], outs["0"]):
        assert not torch.isnan(a).any() and torch.equal(a, r)


def _pipeline_run(monkeypatch, prefetch: bool, overlap: bool, steps: int = 3):
    """Three Adam steps of the 5,5,5/16,16,1 model on alternating batches."""
    from ncnet_amd.engine.trainer import TrunkPrefetcher, make_adam, weak_loss_from_features
    from ncnet_amd.models import ImMatchNet
    import importlib

    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")   # the module, not the re-exported function

    from tests.conftest import set_runtime
    set_runtime(monkeypatch, trunk_prefetch=prefetch, bwd_overlap=overlap)
    torch.manual_seed(0)
    model = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(DEV)
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = make_adam(params, 5e-4)
    g = torch.Generator(device=DEV).manual_seed(7)
    pool = [{"source_image": torch.randn(4, 3, 200, 200, device=DEV, generator=g),
             "target_image": torch.randn(4, 3, 200, 200, device=DEV, generator=g)} for _ in range(2)]
    pre = TrunkPrefetcher(model)
    assert pre.enabled == prefetch
    losses = []
    for it in range(steps):
        opt.zero_grad(set_to_none=True)
        feats = pre.take(pool[it % 2])
        pre.submit(pool[(it + 1) % 2])
        loss = weak_loss_from_features(model, feats)
        loss.backward()
        opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    return torch.stack(losses).cpu(), [p.detach().clone().cpu() for p in params]


def test_pipelined_step_equals_serial(monkeypatch):
    """Trunk prefetch on a side stream + NC weight gradients on a side stream
    must be bit-identical to the serial schedule (same kernels, same order of
    accumulation; only the stream placement differs)."""
    l_ser, p_ser = _pipeline_run(monkeypatch, prefetch=False, overlap=False)
    l_pip, p_pip = _pipeline_run(monkeypatch, prefetch=True, overlap=True)
    assert torch.equal(l_ser, l_pip), (l_ser, l_pip)
    for a, b in zip(p_ser, p_pip):
        assert torch.equal(a, b)


def test_resize_norm_u8_kernel():
    """One-launch batched resize + normalise of packed HWC uint8 images of
    different sizes (csrc/dataprep.hip) vs torch bilinear (align_corners=True)
    + ImageNet normalisation."""
    from ncnet_amd.data.datasets import collate_uint8_pairs, gpu_pair_batch
    from ncnet_amd.data.transforms import gpu_normalize_resize
    g = torch.Generator().manual_seed(5)
    samples = []
    for (h1, w1), (h2, w2) in (((375, 500), (500, 333)), ((300, 300), (481, 322)), ((17, 9), (400, 400))):
        samples.append({"source_image": torch.randint(0, 256, (h1, w1, 3), generator=g, dtype=torch.uint8),
                        "target_image": torch.randint(0, 256, (h2, w2, 3), generator=g, dtype=torch.uint8),
                        "set": 1})
    batch = collate_uint8_pairs(samples)
    out = gpu_pair_batch(batch, DEV, 400, 400)
    for k in ("source_image", "target_image"):
        want = torch.cat([gpu_normalize_resize(s[k].permute(2, 0, 1).unsqueeze(0).to(DEV), 400, 400)
                          for s in samples])
        assert out[k].shape == want.shape
        assert (out[k] - want).abs().max() < 2e-4


def test_debug_build_selftest(capfd):
    """Sanitizer tier: the debug build (NCNET_EXT=debug) reports a failed
    device-side bounds check by printing it (and skipping the access); the
    release build compiles the checks away."""
    from ncnet_amd.ops._ext import ext
    out = torch.zeros(1, dtype=torch.int32, device=DEV)
    r = ext().debug_selftest(out)
    torch.cuda.synchronize()
    text = capfd.readouterr().out
    if os.environ.get("NCNET_EXT") == "debug":
        assert r == 0 and "NCNET_CHECK failed" in text
    else:
        assert r == 1 and "NCNET_CHECK" not in text


@pytest.mark.parametrize("cfg", [None, (3, 4, 6, 7), (2, 3, 16, 20), (5, 2, 9, 11)])
def test_nc_fused_k3_vs_quantized_oracle(cfg):
    """The fused InLoc NeighConsensus kernel (csrc/nc_fused.hip: 1 -> 16 -> 1,
    k = 3, hidden layer in LDS) against the fp64 oracle with bf16 rounding of
    x0, the weights and the hidden activation; cfg = (R, IR, TK, TL) forces
    multi-workgroup splits along j, i and the (k, l) tile (None: the
    production choice, fused_tiles)."""
    import importlib
    from ncnet_amd.engine import quantized_oracle as qo
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(21)
    V, I, J, K, L = 2, 9, 13, 11, 14
    w1 = torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2
    w2 = torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.1
    b1, b2 = torch.rand(16, device=DEV) * 0.1 - 0.03, torch.rand(1, device=DEV) * 0.1
    ws = [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)]
    x0 = torch.rand(V, I, J, K, L, device=DEV).to(torch.bfloat16)
    wts = nc._fused_weights(ws, [b1, b2])
    y = torch.full((V, I, J, K, L), float("nan"), device=DEV)
    tk, tl, R, IR = nc.fused_tiles(V, I, J, K, L) if cfg is None else (cfg[2], cfg[3], cfg[0], cfg[1])
    _ext.ext().nc_fused_k3(x0, *wts, y, R, IR, tk, tl)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    yr = qo.nc_stack(x0.double().unsqueeze(1), [w1.double(), w2.double()], [b1.double(), b2.double()])
    assert relerr(y, yr.squeeze(1)) < 2e-3


@pytest.mark.parametrize("shape", [(1, 7500, 7500), (3, 625, 400), (2, 130, 1852), (1, 64, 256), (4, 625, 625),
                                   (2, 77, 1850), (1, 3, 5)])
@pytest.mark.parametrize("sum_kind", [0, 1, 2])
def test_stats2d_matches_row_and_col_kernels(shape, sum_kind):
    """One-pass row + column statistics (csrc/volume.hip stats2d; 16-byte
    loads, or scalar loads when C % 4 != 0) equal the separate stats_rows /
    stats_cols kernels: max and first argmax exactly (values drawn from a small
    set: many ties), the sums to fp32 rounding."""
    V, R, C = shape
    torch.manual_seed(31)
    x = (torch.randint(0, 50, shape, device=DEV).float() / 7.0 - 3.0).contiguous()
    E = _ext.ext()
    f = dict(dtype=torch.float32, device=DEV)
    out = []
    for fused in (True, False):
        rmx, cmx = torch.empty((V, R), **f), torch.empty((V, C), **f)
        rarg, carg = (torch.empty((V, n), dtype=torch.int32, device=DEV) for n in (R, C))
        rse, cse = torch.empty((V, R), **f), torch.empty((V, C), **f)
        if fused:
            assert E.stats2d(x, rmx, rarg, rse, cmx, carg, cse, sum_kind)
        else:
            E.stats_rows(x, rmx, rarg, rse if sum_kind else None, sum_kind)
            E.stats_cols(x, cmx, carg, cse if sum_kind else None, sum_kind)
        out.append((rmx, rarg, rse, cmx, carg, cse))
    a, b = out
    for i in (0, 1, 3, 4):
        assert torch.equal(a[i], b[i]), i
    if sum_kind:
        for i in (2, 5):
            assert torch.allclose(a[i], b[i], rtol=1e-5, atol=1e-5), (i, (a[i] - b[i]).abs().max())


@pytest.mark.parametrize("k,packed,softmax", [(2, True, True), (2, True, False), (1, False, True), (2, False, True),
                                               (3, "tuple", True), (4, "tuple", False)])
def test_fused_match_candidates_match_op_path(k, packed, softmax, monkeypatch):
    """InLoc pair_matches through stats2d + match_candidates (one launch for
    both directions' candidates, offsets decoded, recentred) against the
    op-by-op corr_to_matches path: identical de-duplicated order and keys,
    coordinates to 1e-6 (linspace rounding).  ``packed="tuple"`` passes the
    unpacked (di, dj, dk, dl) offsets that _fused_candidates packs itself."""
    import ncnet_amd.eval.inloc as inl
    torch.manual_seed(33)
    fs = (9, 12, 9, 12)
    corr = (torch.randint(0, 40, (1, 1) + fs, device=DEV).float() / 9.0).contiguous()
    code = None
    if packed:   # 2-bit fields, each an in-cell offset < k (as the fused pool writes them)
        f4 = torch.randint(0, k, (4, 1, 1) + fs, device=DEV)
        code = ((f4[0] << 6) | (f4[1] << 4) | (f4[2] << 2) | f4[3]).to(torch.uint8)
        if packed == "tuple":
            code = tuple(f4[i].long() for i in range(4))
            assert inl._fused_candidates(corr, code, k, softmax) is not None
            # 2-bit fields cannot hold offsets of a k > 4 pool: op-by-op path
            assert inl._fused_candidates(corr, code, 5, softmax) is None
    if k > 1 and not packed:
        code = None
    got, n_got = inl.pair_matches(corr, code, k, do_softmax=softmax, static=True)
    monkeypatch.setattr(inl, "_fused_candidates", lambda *a, **kw: None)
    want, n_want = inl.pair_matches(corr, code, k, do_softmax=softmax, static=True)
    assert int(n_got) == int(n_want)
    n = int(n_got)
    assert torch.allclose(got[:n], want[:n], atol=1e-6, rtol=0), (got[:n] - want[:n]).abs().max()
    assert torch.equal(got[:n, 4], want[:n, 4])


def test_nc_fused_k3_one_wide_workgroup():
    """The > 80 KB configuration of the fused NC kernel (a 24-plane output
    ring: one 16-wave workgroup per CU, csrc/nc_fused.hip NW = 16) against the
    quantized fp64 oracle."""
    import importlib
    from ncnet_amd.engine import quantized_oracle as qo
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(23)
    V, I, J, K, L = 1, 6, 26, 17, 22
    w1 = torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2
    w2 = torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.1
    b1, b2 = torch.rand(16, device=DEV) * 0.1 - 0.03, torch.rand(1, device=DEV) * 0.1
    x0 = torch.rand(V, I, J, K, L, device=DEV).to(torch.bfloat16)
    wts = nc._fused_weights([ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)], [b1, b2])
    y = torch.full((V, I, J, K, L), float("nan"), device=DEV)
    _ext.ext().nc_fused_k3(x0, *wts, y, 24, 4, 15, 20)      # R = 24, IR = 4, 15 x 20 tiles
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    yr = qo.nc_stack(x0.double().unsqueeze(1), [w1.double(), w2.double()], [b1.double(), b2.double()])
    assert relerr(y, yr.squeeze(1)) < 2e-3


@pytest.mark.parametrize("tiles", [(8, 4, 8, 8), (10, 4, 15, 20), (24, 4, 15, 20)])
def test_nc_fused_k3_last_volume_borders(tiles):
    """The fused NC kernel's out-of-volume gathers issue their load with the
    scalar offset past the volume's buffer range (csrc/nc_fused.hip gather):
    a single volume followed by large non-zero data in the same allocation
    must still see zero padding at every border (the range check covers the
    scalar offset on gfx950; a read past the tensor would show here as a
    large error at the I/J borders)."""
    import importlib
    from ncnet_amd.engine import quantized_oracle as qo
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(29)
    I, J, K, L = 7, 9, 11, 13
    n = I * J * K * L
    big = torch.full((3 * n,), 50.0, device=DEV, dtype=torch.bfloat16)    # poison after the tensor
    big[:n] = torch.rand(n, device=DEV).to(torch.bfloat16)
    x0 = big[:n].view(1, I, J, K, L)
    w1 = torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2
    w2 = torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.1
    b1, b2 = torch.rand(16, device=DEV) * 0.1 - 0.03, torch.rand(1, device=DEV) * 0.1
    wts = nc._fused_weights([ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)], [b1, b2])
    y = torch.full((1, I, J, K, L), float("nan"), device=DEV)
    _ext.ext().nc_fused_k3(x0, *wts, y, *tiles)          # R, IR, TK, TL (runtime, 3200-px static, 16-wave)
    torch.cuda.synchronize()
    yr = qo.nc_stack(x0.double().unsqueeze(1), [w1.double(), w2.double()], [b1.double(), b2.double()])
    assert torch.isfinite(y).all()
    assert relerr(y, yr.squeeze(1)) < 2e-3
    # the border planes alone (where every out-of-volume combo lands)
    for sl in ((slice(None), 0), (slice(None), I - 1), (slice(None), slice(None), 0), (slice(None), slice(None), J - 1)):
        assert relerr(y[sl], yr.squeeze(1)[sl]) < 2e-3, sl


def test_neigh_consensus_fused_symmetric_wrapper():
    """The symmetric InLoc NC (both branches through the fused kernel in one
    launch: cast + transpose into one [2V, ...] input, then the combine)
    against the quantized fp64 oracle of the whole symmetric stack."""
    import importlib
    from ncnet_amd.engine import quantized_oracle as qo
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(22)
    w1 = torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2
    w2 = torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.1
    b1, b2 = torch.rand(16, device=DEV) * 0.1, torch.rand(1, device=DEV) * 0.1
    x = torch.rand(2, 1, 7, 9, 7, 9, device=DEV).to(torch.bfloat16).float()
    with torch.inference_mode():
        y = nc.neigh_consensus_fused(x, [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)],
                                     [b1, b2], symmetric=True)
    yr = qo.neigh_consensus(x.double(), [w1.double(), w2.double()], [b1.double(), b2.double()], symmetric=True)
    assert relerr(y, yr) < 2e-3


def _f8q(t, s):
    """OCP e4m3 rounding at the power-of-two scale s (values returned unscaled, fp64)."""
    return (t.double() * s).float().clamp(-448, 448).to(torch.float8_e4m3fn).double() / s


@pytest.mark.parametrize("cfg", [None, (3, 4, 6, 7), (10, 4, 15, 20), (8, 3, 19, 17), (5, 2, 9, 11)])
def test_nc_fused_k3_f8_vs_quantized_oracle(cfg):
    """The e4m3 fused NC kernel (csrc/nc_fused.hip nc_fused_k3_f8: one MX
    16x16x128 MFMA for taps 0-7 + one 16x16x32 fp8 MFMA for tap 8 per tile and
    layer, register-resident weight fragments) against fp64 math with the same
    e4m3 roundings (x0 * sx, weights * sw, hidden * sh): a wrong lane -> tap /
    channel map shows as an O(1) error, the fp8 quantisation itself cancels.
    cfg = (R, IR, TK, TL); the 3200 px (15 x 20, R 10) and 1600 px (19 x 17,
    R 8) tiles are the compile-time instantiations."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(41)
    V, I, J, K, L = 2, 9, 13, 11, 14
    w1 = torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2
    w2 = torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.1
    b1, b2 = torch.rand(16, device=DEV) * 0.1 - 0.03, torch.rand(1, device=DEV) * 0.1
    ws = [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)]
    # MutualMatching-like input: [0, 1], most entries small
    x0 = (torch.rand(V, I, J, K, L, device=DEV) ** 3).to(torch.bfloat16)
    tens, (sx, inv1, sh, inv2) = nc._fused_weights_f8_build(ws, [b1, b2])
    sw1, sw2 = 1.0 / (inv1 * sx), 1.0 / (inv2 * sh)
    y = torch.full((V, I, J, K, L), float("nan"), device=DEV)
    tk, tl, R, IR = nc.fused_tiles(V, I, J, K, L) if cfg is None else (cfg[2], cfg[3], cfg[0], cfg[1])
    _ext.ext().nc_fused_k3_f8(x0, *tens, y, R, IR, tk, tl, sx, inv1, sh, inv2)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    xq = _f8q(x0, sx).unsqueeze(1)
    h = torch.relu(ref.conv4d(xq, ref.conv4d_weight_from_std(_f8q(w1, sw1))) + b1.double().view(1, -1, 1, 1, 1, 1))
    h = _f8q(h, sh)
    yr = torch.relu(ref.conv4d(h, ref.conv4d_weight_from_std(_f8q(w2, sw2))) + b2.double().view(1, -1, 1, 1, 1, 1))
    # (a hidden value on the other side of an e4m3 rounding boundary in fp32
    # vs fp64 moves by one e4m3 ulp, 6 %: a few such flips, not O(1) errors)
    assert relerr(y, yr.squeeze(1)) < 2e-2 and rel_l2(y, yr.squeeze(1)) < 2e-3
    # and the unquantised fp64 stack: the e4m3 error of the whole NC
    yf = ref.neigh_consensus(x0.double().unsqueeze(1), [w.double() for w in ws], [b1.double(), b2.double()],
                             symmetric=False)
    assert rel_l2(y, yf.squeeze(1)) < 0.05


def _pad_1ch(x5, ks, trans=False):
    """x5 [V, I, J, K, L] (any float dtype) -> padded bf16 planes via pad_planes."""
    V, I, J, K, L = x5.shape
    C = _ext.ext()
    lp, ppl = C.pad_geom(K, L, ks) if not trans else C.pad_geom(I, J, ks)
    n = V * (K * L if trans else I * J)
    y = torch.zeros((n, ppl), dtype=torch.bfloat16, device=DEV)
    C.pad_planes(x5.reshape(V, I * J, K * L).contiguous(), y, *((I, J) if trans else (K, L)), ks, 1 if trans else 0)
    return y


@pytest.mark.parametrize("ks,shape", [(5, (2, 25, 25, 25, 25)), (5, (1, 6, 7, 25, 25)), (5, (1, 3, 11, 25, 25)),
                                      (5, (2, 20, 20, 20, 20)), (5, (1, 7, 3, 20, 20)), (3, (2, 25, 25, 25, 25)),
                                      (3, (1, 4, 9, 25, 25)), (5, (1, 30, 30, 30, 30)), (5, (1, 7, 4, 30, 30))])
@pytest.mark.parametrize("epi", [1, 2])
def test_conv1x16_vs_oracle(ks, shape, epi):
    """1 -> 16 Conv4d on zero-padded 1-channel planes (csrc/conv1x.hip: taps
    gathered by ds_read_b64_tr_b16 from 4 element-shifted LDS copies of each
    plane) vs the fp64 oracle: bias + ReLU forward, and the ReLU-mask epilogue
    of the last layer's data gradient."""
    from ncnet_amd.ops.packing import pack_w1x
    torch.manual_seed(3)
    V, I, J, K, L = shape
    x = torch.rand(V, I, J, K, L, device=DEV).to(torch.bfloat16)
    w = torch.randn(16, 1, ks, ks, ks, ks, device=DEV) * 0.05
    b = torch.randn(16, device=DEV) * 0.1
    m = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    y = torch.full((V, I, J, K, L, 16), float("nan"), dtype=torch.bfloat16, device=DEV)
    ran = _ext.ext().conv1x16(_pad_1ch(x, ks), pack_w1x(w), b if epi == 1 else None, m if epi == 2 else None, y, ks, epi)
    assert ran
    z = ref.conv4d(x.double().unsqueeze(1), ref.conv4d_weight_from_std(bf(w)), None)   # [V, 16, I, J, K, L]
    if epi == 1:
        want = torch.relu(z + b.double().view(1, 16, 1, 1, 1, 1))
    else:
        want = z * (m.double().permute(0, 5, 1, 2, 3, 4) > 0)
    assert relerr(y.permute(0, 5, 1, 2, 3, 4), want) < 1e-2


def test_pad_planes_transposed():
    """pad_planes trans=1 writes the planes of the A<->B-swapped volume."""
    torch.manual_seed(4)
    V, I, J, K, L = 2, 9, 11, 9, 11
    x = torch.randn(V, I, J, K, L, device=DEV)
    a = _pad_1ch(x, 5, trans=True)
    b = _pad_1ch(x.permute(0, 3, 4, 1, 2).contiguous(), 5)
    assert torch.equal(a, b)


@pytest.mark.parametrize("ks,shape,G", [(5, (2, 25, 25, 25, 25), 256), (5, (1, 6, 7, 25, 25), 7),
                                        (5, (1, 3, 11, 25, 25), 64), (5, (1, 5, 5, 25, 25), 1),
                                        (5, (2, 20, 20, 20, 20), 256), (5, (1, 4, 9, 20, 20), 13),
                                        (3, (2, 25, 25, 25, 25), 256), (3, (1, 5, 7, 25, 25), 9),
                                        (5, (1, 30, 30, 30, 30), 256), (5, (1, 4, 9, 30, 30), 13)])
@pytest.mark.parametrize("bias", [True, False])
def test_wgrad1x16_vs_oracle(ks, shape, G, bias):
    """Weight gradient with a 1-channel operand straight from padded planes
    (csrc/conv1x.hip wgrad1x16: tap shift moved into the transposed D read, one
    partial per persistent workgroup, item starts at arbitrary (v, i, j) steps)
    vs autograd of the fp64 oracle, for both uses: the first layer (D = output
    gradient, X1 = input: R = dW) and the Cout = 1 last layer (D = input,
    X1 = output gradient: dW = R with all four kernel axes flipped)."""
    torch.manual_seed(21)
    V, I, J, K, L = shape
    x1 = torch.rand(V, I, J, K, L, device=DEV).to(torch.bfloat16)
    d = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    nt = ks * ks
    part = torch.full((G, nt, 32, 16), float("nan"), device=DEV)
    partb = torch.full((G, 16), float("nan"), device=DEV) if bias else None
    assert _ext.ext().wgrad1x16(d, _pad_1ch(x1, ks), part, partb, ks)
    R = part.sum(0)[:, :nt, :]                                   # [tap, combo, c]
    # first layer: y[co] = conv(x1; W[co, 0]), dL/dy = d  ->  dW[co, 0, di, dj, dk, dl]
    wr = torch.zeros(ks, 16, 1, ks, ks, ks, device=DEV, dtype=torch.float64, requires_grad=True)
    yr = ref.conv4d(x1.double().unsqueeze(1), wr, None)
    (yr * d.double().permute(0, 5, 1, 2, 3, 4)).sum().backward()
    want = ref.conv4d_weight_to_std(wr.grad)[:, 0].reshape(16, nt, nt)      # [co, combo, tap]
    assert relerr(R.permute(2, 1, 0), want) < 1e-4
    # last layer: y = conv(d; W[0, ci]), dL/dy = x1  ->  dW[0, ci, t] = R[2P - t][ci]
    w3 = torch.zeros(ks, 1, 16, ks, ks, ks, device=DEV, dtype=torch.float64, requires_grad=True)
    y3 = ref.conv4d(d.double().permute(0, 5, 1, 2, 3, 4), w3, None)
    (y3 * x1.double().unsqueeze(1)).sum().backward()
    want3 = ref.conv4d_weight_to_std(w3.grad)[0]                               # [ci, di, dj, dk, dl]
    got3 = R.permute(2, 1, 0).reshape(16, ks, ks, ks, ks).flip(1, 2, 3, 4)
    assert relerr(got3, want3) < 1e-4
    if bias:
        assert relerr(partb.sum(0), d.double().sum(dim=(0, 1, 2, 3, 4))) < 1e-4


@pytest.mark.parametrize("symmetric", [True, False])
def test_neigh_consensus_fast1x_matches_ij_path(monkeypatch, symmetric):
    """The training stack 5,5,5 / 16,16,1 at a 25^4 volume on the padded-plane
    1-channel kernels (conv1x16 forward / data gradient, wgrad1x16 for both
    1-channel layers) vs the ij-packed path and the fp64 oracle: output and every
    gradient."""
    import importlib
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(31)
    x = torch.rand(2, 1, 25, 25, 25, 25, device=DEV).to(torch.bfloat16).float()
    ws, bs, cin = [], [], 1
    for k, c in zip((5, 5, 5), (16, 16, 1)):
        ws.append((torch.randn(k, c, cin, k, k, k, device=DEV) * 0.05).to(torch.bfloat16).float())
        bs.append(0.2 + torch.rand(c, device=DEV) * 0.1)
        cin = c
    g = torch.randn(2, 1, 25, 25, 25, 25, device=DEV)
    outs = {}
    for fast in (True, False):
        monkeypatch.setattr(nc, "FAST1X", fast)
        xx = x.clone().requires_grad_(True)
        pw = [w.clone().requires_grad_(True) for w in ws]
        pb = [b.clone().requires_grad_(True) for b in bs]
        assert nc.fast1x_ok(["1in", "16", "1out"], [16, 16, 1], [5, 5, 5], xx, symmetric) == fast
        y = nc.neigh_consensus(xx, pw, pb, [16, 16, 1], symmetric=symmetric)
        (y * g).sum().backward()
        outs[fast] = [y.detach(), xx.grad] + [p.grad for p in pw + pb]
    xr = x.double().requires_grad_(True)
    wr = [w.double().requires_grad_(True) for w in ws]
    br = [b.double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wr, br, symmetric=symmetric)
    (yr * g.double()).sum().backward()
    want = [yr, xr.grad] + [p.grad for p in wr + br]
    names = ["y", "gx", "gw0", "gw1", "gw2", "gb0", "gb1", "gb2"]
    for n, a, b, r in zip(names, outs[True], outs[False], want):
        ea, eb = rel_l2(a, r), rel_l2(b, r)
        assert ea < max(2 * eb, 2e-2), (n, ea, eb)
        assert rel_l2(a, b) < 5e-2, (n, rel_l2(a, b))


def _fast1x_vs_quantized_oracle(symmetric, perturb=None, seed=31, ks=(5, 5, 5), ch=(16, 16, 1), T=25, V=2):
    """The fast training stack on the padded-plane kernels vs the quantized
    fp64 oracle (engine/quantized_oracle.py: bf16 rounding exactly at the
    stored activations, weights and pre-activation gradients).  Returns
    {name: rel L2 error}.  ``perturb``: a function applied to the first layer's
    packed weights (a mutation the check must catch).

    The data are small multiples of powers of two (x in {0, 1}, weights and
    biases k / 8 .. k / 32, |k| <= 2, output gradient k / 16) so every
    pre-activation and every pre-activation gradient is EXACT in fp32: the
    kernels and the oracle then round the same values to bf16 and take the
    same ReLU masks.  With continuous random data a relative error of ~1e-6 in
    fp32 flips ~1e-4 of the masks, and every flip moves a gradient element by
    its full value (an L2 error of sqrt(1e-4) = 1e-2 whatever the kernels do)."""
    import importlib
    from ncnet_amd.engine import quantized_oracle as qo
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    gen = torch.Generator(device=DEV).manual_seed(seed)

    def ints(shape, lo, hi, scale):
        return torch.randint(lo, hi + 1, shape, device=DEV, generator=gen).float() * scale

    x = ints((V, 1, T, T, T, T), 0, 1, 1.0)
    ws, bs, cin = [], [], 1
    for li, (k, c) in enumerate(zip(ks, ch)):
        sc = 2.0 ** (-3 if li == 0 else -5)
        ws.append(ints((k, c, cin, k, k, k), -2, 2, sc))
        bs.append(ints((c,), -2, 2, sc))
        cin = c
    g = ints((V, 1, T, T, T, T), -1, 1, 2.0 ** -4)
    xx = x.clone().requires_grad_(True)
    pw = [w.clone().requires_grad_(True) for w in ws]
    pb = [b.clone().requires_grad_(True) for b in bs]
    kinds = nc.layer_kinds(list(ch), list(ks))
    assert nc.fast1x_ok(kinds, list(ch), list(ks), xx, symmetric)
    orig = nc.pack_w1x
    if perturb is not None:
        calls = []

        def mutated(w_std):
            p = orig(w_std)
            if not calls:                 # the first layer's forward packing only
                p = perturb(p)
            calls.append(1)
            return p
        nc.pack_w1x = mutated
    try:
        y = nc.neigh_consensus(xx, pw, pb, list(ch), symmetric=symmetric)
        (y * g).sum().backward()
    finally:
        nc.pack_w1x = orig
    got = [y.detach(), xx.grad] + [p.grad for p in pw + pb]
    xr = x.double().requires_grad_(True)
    wr = [ref.conv4d_weight_to_std(w.double()).requires_grad_(True) for w in ws]
    br = [b.double().requires_grad_(True) for b in bs]
    yr = qo.neigh_consensus(xr, wr, br, symmetric=symmetric)
    (yr * g.double()).sum().backward()
    want = [yr, xr.grad] + [ref.conv4d_weight_from_std(p.grad) for p in wr] + [p.grad for p in br]
    names = ["y", "gx"] + [f"gw{i}" for i in range(len(ws))] + [f"gb{i}" for i in range(len(ws))]
    # (diagnostic) the unrounded fp64 reference: the quantized oracle must sit
    # ~1e-3 (y) .. ~1e-1 (gradients) from it, the kernels ~1e-3 from the oracle
    x2 = x.double().requires_grad_(True)
    w2 = [w.double().requires_grad_(True) for w in ws]
    b2 = [b.double().requires_grad_(True) for b in bs]
    y2 = ref.neigh_consensus(x2, w2, b2, symmetric=symmetric)
    (y2 * g.double()).sum().backward()
    plain = [y2, x2.grad] + [p.grad for p in w2 + b2]
    print("kernels vs fp64 ref:", {n: f"{rel_l2(a, r):.1e}" for n, a, r in zip(names, got, plain)},
          "oracle vs fp64 ref:", {n: f"{rel_l2(a, r):.1e}" for n, a, r in zip(names, want, plain)})
    return {n: rel_l2(a, r) for n, a, r in zip(names, got, want)}


@pytest.mark.parametrize("ks,ch,T,V", [((5, 5, 5), (16, 16, 1), 20, 2), ((3, 3), (16, 1), 25, 2),
                                       ((5, 5, 5), (16, 16, 1), 30, 1)])
def test_fast1x_other_configs_vs_quantized_oracle(ks, ch, T, V):
    """The fast training stack at --image_size 320 (20^4 volumes), 480 (30^4)
    and the IVD recipe (NC 3,3 / 16,1 at 400 px) vs the quantized fp64 oracle."""
    errs = _fast1x_vs_quantized_oracle(True, ks=ks, ch=ch, T=T, V=V)
    print(f"fast1x {ks}/{ch} at {T}^4 vs quantized oracle:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert max(errs.values()) < 1e-3, errs


@pytest.mark.parametrize("symmetric", [True, False])
def test_fast1x_stack_vs_quantized_oracle(symmetric):
    """Output and every gradient of the fast training stack (conv1x16,
    conv16v4 forward / data gradient, wgrad16v4, wgrad1x16, the Cout=1 block
    forward) within 1e-3 of the quantized fp64 oracle: what remains is fp32
    accumulation order and the rare bf16 rounding-boundary flip."""
    errs = _fast1x_vs_quantized_oracle(symmetric)
    print("fast1x vs quantized oracle:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert max(errs.values()) < 1e-3, errs


def test_fast1x_oracle_check_catches_one_tap():
    """Mutation check of the test above: one (dk, dl) tap of one plane offset of
    the first layer's conv1x16 weights, scaled by 1.5 in the packed operand the
    kernel reads, must push the forward error far past the 1e-3 tolerance."""
    def perturb(p):                       # p [k*k planes, 64 lanes, 8]
        p = p.clone()
        p[12, 0:16, 3] *= 1.5             # plane (2, 2), tap 3, all 16 output channels
        return p
    errs = _fast1x_vs_quantized_oracle(True, perturb=perturb)
    print("mutated conv1x16 tap:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert errs["y"] > 1e-2, errs


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw", [(50, 50), (37, 61)])
def test_maxpool_bias_act_matches_separate_passes(dtype, hw):
    """The trunk stem's fused bias + ReLU + 3x3/2 max-pool (csrc/epilogue.hip)
    equals bias_act followed by PyTorch's max_pool2d bit for bit (the rounded
    activation is monotonic, so it commutes with max)."""
    torch.manual_seed(41)
    x = torch.randn(3, 64, *hw, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, device=DEV)
    want = torch.nn.functional.max_pool2d(torch.relu(x.float() + b.view(1, -1, 1, 1)).to(dtype), 3, 2, 1)
    ho, wo = want.shape[2:]
    y = torch.empty((3, 64, ho, wo), dtype=dtype, device=DEV, memory_format=torch.channels_last)
    _ext.ext().maxpool_bias_act(x, b, y, 3, 2, 1, 1)
    assert torch.equal(y, want)
