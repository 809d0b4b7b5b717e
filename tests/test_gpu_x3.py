"""GPU: the fused bf16x3 ("fp32-accurate") training NeighConsensus
(ops/neigh_consensus.py NeighConsensusX3FusedFn on csrc/conv4d_fwd.hip EPI_X3)
against autograd of the fp64 reference algorithm.  25 x 25 planes run the
conv16v4 kernel with the three phases, smaller planes the conv16v2 ones."""
import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _params(ks, ch, seed, masked=False):
    """masked: positive weights, negative biases -- the ReLU masks are active but
    no gradient sum cancels (with random signs the first layer's weight / bias
    gradients cancel ~300x and any fp32-class method shows ~5e-3 there)."""
    g = torch.Generator().manual_seed(seed)
    ws, bs, cin = [], [], 1
    for k, c in zip(ks, ch):
        w = torch.randn(c, cin, k, k, k, k, generator=g) * (0.5 / (cin * k ** 4) ** 0.5)
        b = torch.rand(c, generator=g) * 0.1
        if masked:
            w = w.abs() * 2
            b = b - 2 * w.sum(dim=(1, 2, 3, 4, 5)) * 0.25
        ws.append(ref.conv4d_weight_from_std(w).cuda().requires_grad_(True))
        bs.append(b.cuda().requires_grad_(True))
        cin = c
    return ws, bs


@pytest.mark.parametrize("ks,ch,shape", [((5, 5, 5), (16, 16, 1), (1, 1, 25, 25, 25, 25)),
                                         ((5, 5, 5), (16, 16, 1), (2, 1, 9, 7, 9, 7)),
                                         ((3, 3), (16, 1), (2, 1, 8, 11, 8, 11)),
                                         ((3, 3, 3), (10, 10, 1), (1, 1, 6, 6, 6, 6))])
def test_x3_fused_matches_fp64(ks, ch, shape):
    from ncnet_amd.ops.neigh_consensus import neigh_consensus
    torch.manual_seed(7)
    ws, bs = _params(ks, ch, 11, masked=True)
    # x requires grad: the input gradient (three split data-gradient convs and
    # the symmetric fold gx[:V] + gx[V:]^T) runs with --fe_finetune_params
    x = torch.rand(shape, device="cuda").requires_grad_(True)
    n0 = _ext.DISPATCH["nc_x3_fused"]
    y = neigh_consensus(x, ws, bs, list(ch), symmetric=True, precision="fp32")
    assert _ext.DISPATCH["nc_x3_fused"] == n0 + 1
    gy = torch.rand_like(y)
    (y * gy).sum().backward()
    got = [x.grad.clone()]
    for w, b in zip(ws, bs):
        got += [w.grad.clone(), b.grad.clone()]
    xr = x.detach().double().requires_grad_(True)
    wd = [w.detach().double().requires_grad_(True) for w in ws]
    bd = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wd, bd, True)
    (yr * gy.double()).sum().backward()
    want = [xr.grad]
    for w, b in zip(wd, bd):
        want += [w.grad, b.grad]
    errs = {"y": rl2(y, yr)}
    errs.update({("gx" if i == 0 else f"g{i - 1}"): rl2(a, b) for i, (a, b) in enumerate(zip(got, want))})
    print("x3 fused errors:", {k: f"{v:.1e}" for k, v in errs.items()})
    # bf16x3 keeps ~16 mantissa bits per operand: ~1e-5 relative, vs ~1e-2 for bf16
    assert max(errs.values()) < 2e-4, errs


def _split(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


@pytest.mark.parametrize("grp,plane,epi", [(2, 25, 1), (2, 25, 2), (0, 25, 1), (0, 25, 2), (0, 9, 1), (0, 9, 2),
                                           (2, 9, 2)])
def test_conv16_x3_kernel_vs_emulator(grp, plane, epi):
    """One conv16_fwd_x3 launch (group-plane or full (di, dj) sum; bias+ReLU or
    ReLU-mask epilogue) against the fp64 emulator: hi + lo to ~1e-5."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from tests import emu_ext
    torch.manual_seed(3)
    ks = 5
    V, I, J = 2, 6, 5
    shp = (V, I, J, plane, plane)
    xs = (grp,) if grp else ()
    x = torch.randn(xs + shp + (16,), device="cuda")
    xh, xl = _split(x)
    from ncnet_amd.ops.packing import pack_w16, pack_w16_planes
    if grp:
        w = torch.randn(grp, 16, 16, ks, ks, device="cuda") * 0.05
        pack = pack_w16_planes
    else:
        w = torch.randn(16, 16, ks, ks, ks, ks, device="cuda") * 0.05
        pack = pack_w16
    whi = w.to(torch.bfloat16).float()
    wp2 = torch.stack((pack(whi), pack(w - whi))).contiguous()
    bias = torch.rand(16, device="cuda") * 0.1 if epi == 1 else None
    m = torch.randn(shp + (16,), device="cuda").to(torch.bfloat16) if epi == 2 else None
    yh = torch.empty(shp + (16,), dtype=torch.bfloat16, device="cuda")
    yl = torch.empty_like(yh)
    _ext.ext().conv16_fwd_x3(xh, xl, wp2, bias, m, yh, yl, ks, epi)
    eh = torch.empty(shp + (16,), dtype=torch.float64)
    el = torch.empty_like(eh)
    emu_ext.conv16_fwd_x3(xh.cpu(), xl.cpu(), wp2.cpu(), None if bias is None else bias.cpu(),
                          None if m is None else m.cpu(), eh, el, ks, epi)
    got = yh.double().cpu() + yl.double().cpu()
    want = eh + el
    err = rl2(got, want)
    print("conv16_fwd_x3 error", err)
    assert err < 2e-5, err


def test_x3_fused_matches_per_conv_path():
    """Random-sign weights: the fused kernels reproduce the per-conv bf16x3
    path (NeighConsensusX3Fn, which learns like the fp32 reference,
    profiles/r2_quality) to ~1e-5 in the output and every gradient."""
    from ncnet_amd.ops.neigh_consensus import NeighConsensusX3Fn, NeighConsensusX3FusedFn, layer_kinds
    ks, ch = (5, 5, 5), (16, 16, 1)
    ws, bs = _params(ks, ch, 11)
    torch.manual_seed(7)
    x = torch.rand(2, 1, 9, 7, 9, 7, device="cuda").requires_grad_(True)
    kinds = tuple(layer_kinds(list(ch), list(ks)))
    params = []
    for w, b in zip(ws, bs):
        params += [w, b]
    outs = []
    for fn in (lambda t: NeighConsensusX3FusedFn.apply(t, kinds, ch, *params),
               lambda t: NeighConsensusX3Fn.apply(t, True, kinds, ch, *params)):
        for p in params:
            p.grad = None
        x.grad = None
        y = fn(x)
        torch.manual_seed(8)
        (y * torch.randn_like(y)).sum().backward()
        outs.append([y.detach(), x.grad.clone()] + [p.grad.clone() for p in params])
    errs = [rl2(a, b) for a, b in zip(*outs)]
    assert max(errs) < 1e-4, errs
