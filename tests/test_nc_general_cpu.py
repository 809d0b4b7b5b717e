"""The HIP NeighConsensus / Conv4d orchestration (channel blocks of 16, ij
encoding of 1-channel operands, kernel sizes 1/3/5/7, symmetric branches,
side-stream-free CPU run) against autograd of the fp64 reference algorithm,
with the kernels replaced by the exact CPU emulator in tests/emu_ext.py.
Catches packing / block / gradient-routing bugs on CPU; the GPU tests
(test_gpu_nc_stages.py) run the same configurations on the real kernels."""
import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.conv4d import Conv4dFn
from ncnet_amd.ops.neigh_consensus import NeighConsensusFn, layer_kinds
from tests.emu_ext import EmuExt


@pytest.fixture
def emu(monkeypatch):
    monkeypatch.setattr(_ext, "_C", EmuExt)
    monkeypatch.setattr(_ext, "load", lambda: EmuExt)
    yield


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _params(ks, ch, mode, seed=0):
    g = torch.Generator().manual_seed(seed)
    ws, bs, cin = [], [], 1
    for k, c in zip(ks, ch):
        w = torch.randn(c, cin, k, k, k, k, generator=g) * (0.5 / (cin * k ** 4) ** 0.5)
        b = torch.rand(c, generator=g) * 0.1
        if mode != "mixed":
            w = w.abs() * 2
        if mode == "masked":              # pre-activations straddle 0: the ReLU masks matter
            b = b - 2 * w.sum(dim=(1, 2, 3, 4, 5)) * 0.25
        ws.append(ref.conv4d_weight_from_std(w).requires_grad_(True))
        bs.append(b.requires_grad_(True))
        cin = c
    return ws, bs


CONFIGS = [
    ((5, 5, 5), (16, 16, 1)),      # PF-Pascal / IVD training stack
    ((3, 3), (16, 1)),             # InLoc stack
    ((3, 3, 3), (10, 10, 1)),      # reference default kwargs (lib/model.py:201-202)
    ((5, 5), (32, 1)),             # two output blocks, then a two-block Cout=1 layer
    ((7, 3), (16, 1)),             # KS = 7
    ((1, 3), (16, 1)),             # KS = 1
    ((3, 3), (20, 24)),            # stack not ending in one channel, 2 x 2 blocks
    ((3,), (1,)),                  # 1 -> 1
    ((3, 3, 3), (16, 1, 16)),      # 1-channel layer mid-stack
]


@pytest.mark.parametrize("ks,ch", CONFIGS)
@pytest.mark.parametrize("symmetric,shape", [(True, (2, 1, 5, 4, 5, 4)), (True, (1, 1, 4, 5, 3, 6)),
                                             (False, (2, 1, 4, 5, 3, 4))])
@pytest.mark.parametrize("mode", ["positive", "masked", "mixed"])
def test_nc_stack_matches_oracle(emu, ks, ch, symmetric, shape, mode):
    """positive: all-positive weights / gradients (no ReLU mask flips, no
    cancellation: bf16 storage costs < 1%, so any routing error shows);
    masked: positive weights, negative biases (masks active, few bf16 flips);
    mixed: random signs (cancelling sums amplify bf16 rounding: loose bound)."""
    torch.manual_seed(1)
    kinds = layer_kinds(list(ch), list(ks))
    assert kinds is not None
    positive = mode != "mixed"
    ws, bs = _params(ks, ch, mode)
    x = torch.rand(shape).to(torch.bfloat16).float()
    xa = x.clone().requires_grad_(True)
    params = []
    for w, b in zip(ws, bs):
        params += [w, b]
    y = NeighConsensusFn.apply(xa, symmetric, tuple(kinds), tuple(ch), *params)
    gy = torch.rand_like(y) if positive else torch.randn_like(y)
    (y * gy).sum().backward()
    got = [xa.grad] + [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    xr = x.double().requires_grad_(True)
    wd = [w.detach().double().requires_grad_(True) for w in ws]
    bd = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wd, bd, symmetric)
    (yr * gy.double()).sum().backward()
    want = [xr.grad]
    for w, b in zip(wd, bd):
        want += [w.grad, b.grad]
    assert y.shape == yr.shape
    errs = {"y": rl2(y, yr)}
    errs.update({f"g{i}": rl2(a, b) for i, (a, b) in enumerate(zip(got, want))})
    assert max(errs.values()) < {"positive": 1e-2, "masked": 3e-2, "mixed": 3e-1}[mode], errs


@pytest.mark.parametrize("cin,cout,ks", [(1, 16, 5), (16, 1, 3), (16, 16, 3), (10, 20, 3), (33, 5, 3), (1, 1, 7),
                                         (16, 16, 1), (3, 17, 5)])
def test_conv4d_module_matches_oracle(emu, cin, cout, ks):
    torch.manual_seed(2)
    x = torch.rand(2, cin, 4, 5, 4, 3).to(torch.bfloat16).float()
    w = ref.conv4d_weight_from_std(torch.randn(cout, cin, ks, ks, ks, ks) * 0.1).requires_grad_(True)
    b = (torch.rand(cout) * 0.1).requires_grad_(True)
    xa = x.clone().requires_grad_(True)
    y = Conv4dFn.apply(xa, w, b)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    xr = x.double().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    br = b.detach().double().requires_grad_(True)
    yr = ref.conv4d(xr, wr, br)
    (yr * g.double()).sum().backward()
    errs = {"y": rl2(y, yr), "gx": rl2(xa.grad, xr.grad), "gw": rl2(w.grad, wr.grad), "gb": rl2(b.grad, br.grad)}
    assert max(errs.values()) < 2e-2, errs


def test_even_kernel_raises_on_gpu_policy(runtime):
    """No silent fallback: an even kernel size has no HIP kernel; the GPU
    dispatcher must raise unless NCNET_ALLOW_TORCH_FALLBACK=1."""
    assert layer_kinds([16, 1], [4, 3]) is None
    runtime(allow_torch_fallback=False)
    with pytest.raises(NotImplementedError):
        _ext.torch_fallback("test")
    runtime(allow_torch_fallback=True)
    before = _ext.DISPATCH["torch_fallback"]
    _ext.torch_fallback("test")
    assert _ext.DISPATCH["torch_fallback"] == before + 1


@pytest.mark.parametrize("ks,ch", [((5, 5, 5), (16, 16, 1)), ((3, 3), (16, 1)), ((3, 3), (20, 24))])
def test_nc_x3_fp32_accurate(emu, ks, ch):
    """precision='fp32' (bf16x3 split on the bf16 kernels) matches the fp64
    oracle to ~1e-4 -- two orders tighter than the bf16 stack."""
    from ncnet_amd.ops.neigh_consensus import neigh_consensus_x3
    torch.manual_seed(3)
    ws, bs = _params(ks, ch, "masked")
    x = torch.rand(2, 1, 5, 4, 5, 4)
    with torch.no_grad():
        y = neigh_consensus_x3(x, [w.detach() for w in ws], [b.detach() for b in bs], list(ch), True)
        yr = ref.neigh_consensus(x.double(), [w.detach().double() for w in ws], [b.detach().double() for b in bs], True)
    assert rl2(y, yr) < 3e-4


@pytest.mark.parametrize("ks,ch", [((5, 5, 5), (16, 16, 1)), ((3, 3), (16, 1)), ((3, 3), (20, 24))])
def test_nc_x3_training_gradients(emu, ks, ch):
    """The fp32-accurate training NC (bf16x3 forward, data and weight gradients)
    matches autograd of the fp64 oracle to ~1e-4 (mixed-sign weights)."""
    from ncnet_amd.ops.neigh_consensus import NeighConsensusX3Fn
    torch.manual_seed(4)
    ws, bs = _params(ks, ch, "mixed")
    x = torch.rand(2, 1, 4, 5, 4, 5)
    xa = x.clone().requires_grad_(True)
    params = []
    for w, b in zip(ws, bs):
        params += [w, b]
    y = NeighConsensusX3Fn.apply(xa, True, tuple(layer_kinds(list(ch), list(ks))), tuple(ch), *params)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    got = [xa.grad] + [p.grad.clone() for p in params]
    xr = x.double().requires_grad_(True)
    wd = [w.detach().double().requires_grad_(True) for w in ws]
    bd = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wd, bd, True)
    (yr * gy.double()).sum().backward()
    want = [xr.grad]
    for w, b in zip(wd, bd):
        want += [w.grad, b.grad]
    errs = {"y": rl2(y, yr)}
    errs.update({f"g{i}": rl2(a, b) for i, (a, b) in enumerate(zip(got, want))})
    assert max(errs.values()) < 1e-3, errs


@pytest.mark.parametrize("ks,ch", [((5, 5, 5), (16, 16, 1)), ((3, 3), (16, 1)), ((3, 3, 3), (10, 10, 1))])
def test_nc_x3_fused_training_gradients(emu, ks, ch):
    """The fused bf16x3 training NC (one kernel per conv with the three phases,
    split hi / lo activations and gradients) against autograd of the fp64
    oracle, through the dispatcher (precision='fp32', parameters requiring grad)."""
    from ncnet_amd.ops.neigh_consensus import neigh_consensus
    torch.manual_seed(5)
    ws, bs = _params(ks, ch, "mixed")
    x = torch.rand(2, 1, 5, 4, 5, 4)
    xa = x.clone().requires_grad_(True)
    n0 = _ext.DISPATCH["nc_x3_fused"]
    old = _ext.use_hip
    _ext.use_hip = lambda t: True
    try:
        y = neigh_consensus(xa, ws, bs, list(ch), symmetric=True, precision="fp32")
    finally:
        _ext.use_hip = old
    assert _ext.DISPATCH["nc_x3_fused"] == n0 + 1
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    got = [xa.grad]
    for w, b in zip(ws, bs):
        got += [w.grad.clone(), b.grad.clone()]
    xr = x.double().requires_grad_(True)
    wd = [w.detach().double().requires_grad_(True) for w in ws]
    bd = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wd, bd, True)
    (yr * gy.double()).sum().backward()
    want = [xr.grad]
    for w, b in zip(wd, bd):
        want += [w.grad, b.grad]
    errs = {"y": rl2(y, yr)}
    errs.update({f"g{i}": rl2(a, b) for i, (a, b) in enumerate(zip(got, want))})
    assert max(errs.values()) < 1e-3, errs
