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
                                         ((5, 5, 5), (16, 16, 1), (1, 1, 20, 20, 20, 20)),
                                         ((5, 5, 5), (16, 16, 1), (1, 1, 30, 30, 30, 30)),
                                         ((3, 3), (16, 1), (1, 1, 25, 25, 25, 25)),
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
    # 25 x 25 / 20 x 20 planes: the 1-channel layers on conv1x16's bf16x3 mode and wgrad1x16
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


def _pairs(t_nhwc):
    """fp32 [N, H, W, C] -> bf16 [N, H, W, 2C] = [hi | lo]."""
    hi = t_nhwc.to(torch.bfloat16)
    lo = (t_nhwc - hi.float()).to(torch.bfloat16)
    return torch.cat((hi, lo), -1).contiguous()


def _unpair(p):
    c = p.shape[-1] // 2
    return p[..., :c].double() + p[..., c:].double()


@pytest.mark.parametrize("cin,cout,k,stride,pad,res,relu,shape", [
    (256, 256, 3, 1, 1, False, True, (3, 25, 25)), (1024, 256, 1, 1, 0, False, True, (2, 25, 25)),
    (256, 1024, 1, 1, 0, True, True, (2, 25, 25)), (64, 64, 3, 1, 1, False, True, (2, 37, 29)),
    (128, 128, 3, 2, 1, False, True, (2, 50, 50)), (512, 1024, 1, 2, 0, False, False, (1, 50, 50))])
def test_conv2d_x3_vs_fp64(cin, cout, k, stride, pad, res, relu, shape):
    """conv2d_nhwc_v3 X3 mode: [hi | lo] bf16 pairs in and out, acc = X_hi W_hi +
    X_lo W_hi + X_hi W_lo, fp32 bias / residual / ReLU: the fp32 conv to ~1e-5."""
    C = _ext.ext()
    torch.manual_seed(5)
    n, h, w = shape
    x = torch.randn(n, h, w, cin, device="cuda")
    wt = torch.randn(cout, cin, k, k, device="cuda") * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, device="cuda") * 0.1
    wcl = wt.permute(0, 2, 3, 1)
    whi = wcl.to(torch.bfloat16)
    w3 = torch.cat((whi, whi, (wcl - whi.float()).to(torch.bfloat16)), -1).contiguous()
    xp = _pairs(x)
    want = torch.nn.functional.conv2d(_unpair(xp).permute(0, 3, 1, 2), wt.double(), b.double(), stride, pad)
    want = want.permute(0, 2, 3, 1)
    r = None
    if res:
        rr = torch.randn(want.shape, device="cuda")
        r = _pairs(rr)
        want = want + _unpair(r)
    if relu:
        want = torch.relu(want)
    y = torch.full(tuple(want.shape[:3]) + (2 * cout,), float("nan"), dtype=torch.bfloat16, device="cuda")
    C.conv2d_nhwc_x3(xp, w3, b, r, y, stride, pad, 1 if relu else 0)
    err = rl2(_unpair(y), want)
    print("conv2d x3 error", err)
    assert err < 3e-5, err


def test_trunk_x3_plan_vs_fp64():
    """The bf16x3 trunk plan (FrozenResNetPlanX3: stem im2col GEMM, split
    max-pool, every bottleneck conv on the X3 kernel) against the folded trunk
    evaluated in fp64: fp32-class agreement, and no MIOpen fp32 conv involved."""
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.models.backbones import FrozenResNetPlanX3
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], nc_precision="fp32").cuda().eval()
    fe = m.FeatureExtraction
    x = torch.randn(2, 3, 160, 192, device="cuda")
    with torch.no_grad():
        got = fe.trunk_forward(x, torch.float32)
        assert isinstance(fe._plan_obj, FrozenResNetPlanX3)
        got2 = fe.trunk_forward(x, torch.float32)           # graph replay
        want = fe._folded_trunk().double()(x.double())
        fe._folded = None                                    # (the fp64 copy is not the cached trunk)
    err = rl2(got, want)
    print("x3 trunk vs fp64:", err, "bf16 trunk would be ~1e-2")
    assert torch.equal(got, got2)
    assert err < 1e-4, err


def test_trunk_x3_vs_miopen_fp32():
    """the fp32 trunk modes side by side.  The evaluation default
    (nc_precision 'bf16' / fp32 eval: ``fp32_trunk == 'miopen'``) runs true fp32
    MIOpen convs, the reference's numerics; the bf16x3 plan (``'x3'``, the
    default of nc_precision='fp32' training only) agrees with it to the x3
    split's ~2^-16 operand accuracy: features within 1e-4 relative L2 and
    argmax-over-channels decisions almost everywhere identical."""
    from ncnet_amd import config as _config
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1]).cuda().eval()
    fe = m.FeatureExtraction
    assert fe.fp32_trunk == "miopen"
    x = torch.randn(2, 3, 160, 192, device="cuda")
    with torch.no_grad():
        ref32 = fe.trunk_forward(x, torch.float32)
        want = fe._folded_trunk().double()(x.double())
        fe._folded = None
        with _config.override(trunk_fp32="x3"):
            got = fe.trunk_forward(x, torch.float32)
    e_x3, e_mi, e_pair = rl2(got, want), rl2(ref32, want), rl2(got, ref32)
    print(f"trunk vs fp64: x3 {e_x3:.2e}, miopen fp32 {e_mi:.2e}; x3 vs miopen {e_pair:.2e}")
    assert e_mi < 1e-5, e_mi
    assert e_pair < 1e-4, e_pair
    same = (got.argmax(1) == ref32.argmax(1)).float().mean().item()
    assert same > 0.99, same


@pytest.mark.parametrize("ks,ch,shape", [((5, 5, 5), (16, 16, 1), (1, 1, 25, 25, 25, 25)),
                                         ((3, 3), (16, 1), (1, 1, 25, 25, 25, 25))])
def test_mixed_backward_matches_x3_ablation(ks, ch, shape):
    """precision='mixed' (NeighConsensusMixedFn: the bf16x3 forward, a bf16
    backward on the padded-plane training kernels with the (X_lo, G) weight-
    gradient products) against the bf16x3 stack run with the same stages
    dropped to bf16 (x3_ablation nc_grad + nc_w_bwd: mathematically the same
    products): identical forward, gradients within the summation-order noise."""
    from ncnet_amd.ops.neigh_consensus import neigh_consensus, x3_ablation
    torch.manual_seed(8)
    x0 = torch.rand(shape, device="cuda")
    outs = {}
    for mode in ("mixed", "ablation"):
        ws, bs = _params(ks, ch, 12)
        x = x0.clone().requires_grad_(True)
        if mode == "mixed":
            n0 = _ext.DISPATCH["nc_mixed"]
            y = neigh_consensus(x, ws, bs, list(ch), symmetric=True, precision="mixed")
            assert _ext.DISPATCH["nc_mixed"] == n0 + 1
        else:
            with x3_ablation(["nc_grad", "nc_w_bwd"]):
                y = neigh_consensus(x, ws, bs, list(ch), symmetric=True, precision="fp32")
        gy = torch.rand(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        with x3_ablation(["nc_grad", "nc_w_bwd"] if mode == "ablation" else []):
            (y * gy).sum().backward()
        outs[mode] = [y.detach()] + [x.grad] + [t.grad for pair in zip(ws, bs) for t in pair]
    errs = [rl2(a, b) for a, b in zip(outs["mixed"], outs["ablation"])]
    print("mixed vs ablation:", [f"{e:.1e}" for e in errs])
    assert outs["mixed"][0].abs().max() > 0 and all(t.abs().max() > 0 for t in outs["mixed"][1:])
    assert errs[0] == 0.0, errs
    assert max(errs[1:]) < 2e-3, errs
