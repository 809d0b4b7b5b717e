"""kl kernels (csrc/conv4d_kl.hip) vs the fp64 Conv4d oracle on an MI355X.

Inputs are rounded to the operand dtype first (bf16 / OCP fp8) and the oracle
runs in fp64 on those values.
"""
import importlib

import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"

KL_SHAPES = [(5, (2, 25, 25, 25, 25)), (3, (2, 37, 50, 37, 50)), (3, (1, 7, 9, 30, 61)), (5, (1, 6, 5, 26, 29))]


def bf(x):
    return x.to(torch.bfloat16).double()


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("ks,shape", KL_SHAPES)
def test_conv1to16_kl(ks, shape):
    """1 -> 16: bias+ReLU (bf16 and fp8 out) and the ReLU-mask epilogue."""
    from ncnet_amd.ops.packing import pack_kl_in
    torch.manual_seed(11)
    V, I, J, K, L = shape
    x = torch.rand(V, I, J, K, L, device=DEV)
    w = torch.randn(16, 1, ks, ks, ks, ks, device=DEV) * 0.1
    b = torch.randn(16, device=DEV) * 0.1
    xb = x.to(torch.bfloat16).contiguous()
    conv = ref.conv4d(bf(x).unsqueeze(1), ref.conv4d_weight_from_std(bf(w)))
    yr = torch.relu(conv + b.double().view(1, 16, 1, 1, 1, 1))
    y = torch.empty(V, I, J, K, L, 16, device=DEV, dtype=torch.bfloat16)
    _ext.ext().conv1to16_kl(xb, pack_kl_in(w), b, None, y, ks, 1)
    assert relerr(y.permute(0, 5, 1, 2, 3, 4), yr) < 1e-2
    y8 = torch.empty(V, I, J, K, L, 16, device=DEV, dtype=torch.float8_e4m3fn)
    _ext.ext().conv1to16_kl(xb, pack_kl_in(w), b, None, y8, ks, 1)
    assert rel_l2(y8.float().permute(0, 5, 1, 2, 3, 4), yr) < 5e-2
    m = torch.randn(V, I, J, K, L, 16, device=DEV).to(torch.bfloat16)
    ym = torch.empty_like(m)
    _ext.ext().conv1to16_kl(xb, pack_kl_in(w), None, m, ym, ks, 2)
    ymr = conv * (m.permute(0, 5, 1, 2, 3, 4).double() > 0)
    assert relerr(ym.permute(0, 5, 1, 2, 3, 4), ymr) < 1e-2


@pytest.mark.parametrize("ks,shape", KL_SHAPES)
@pytest.mark.parametrize("f8", [False, True])
def test_conv16to1_kl(ks, shape, f8):
    """16 -> 1 (in-LDS combo shift-sum), bf16 and fp8 operands, fused bias+ReLU."""
    from ncnet_amd.ops.neigh_consensus import _fp8_weights
    from ncnet_amd.ops.packing import pack_kl_out
    torch.manual_seed(12)
    V, I, J, K, L = shape
    x = torch.rand(V, 16, I, J, K, L, device=DEV)
    w = torch.randn(1, 16, ks, ks, ks, ks, device=DEV) * 0.05
    b = torch.full((1,), 0.3, device=DEV)
    xcl = x.permute(0, 2, 3, 4, 5, 1).contiguous()
    y = torch.empty(V, I, J, K, L, device=DEV)
    if f8:
        xq = xcl.to(torch.float8_e4m3fn)
        wq, osc = _fp8_weights(pack_kl_out(w))
        _ext.ext().conv16to1_kl(xq, wq, b, y, ks, 1, osc)
        xr = xq.double().permute(0, 5, 1, 2, 3, 4)
        wr = _unpack_kl_out(wq.double() * osc, ks)          # the exact fp8 weight values used
        # the same fp8 values through the bf16 kernel (e4m3 is a subset of bf16)
        yb = torch.empty_like(y)
        _ext.ext().conv16to1_kl(xq.to(torch.bfloat16), (wq.float() * osc).to(torch.bfloat16), b, yb, ks, 1, 1.0)
        assert relerr(y, yb) < 1e-4
    else:
        _ext.ext().conv16to1_kl(xcl.to(torch.bfloat16), pack_kl_out(w), b, y, ks, 1, 1.0)
        xr = bf(x)
        wr = bf(w)
    yr = torch.relu(ref.conv4d(xr, ref.conv4d_weight_from_std(wr), b.double()))[:, 0]
    assert relerr(y, yr) < 5e-3


def _unpack_kl_out(wl, ks):
    """Inverse of pack_kl_out: [k*k+1, NCT, 16, 16] -> [1, 16, k, k, k, k]."""
    nt = ks * ks
    t = wl[:nt].reshape(nt, -1, 16)[:, :nt]                  # [plane (di,dj), combo (dk,dl), c]
    return t.permute(2, 0, 1).reshape(1, 16, ks, ks, ks, ks)


def test_kl_rejects_bad_shapes():
    """The bindings validate shapes before launching (a malformed call must not reach the GPU)."""
    from ncnet_amd.ops.packing import pack_kl_in, pack_kl_out
    x = torch.zeros(1, 4, 4, 5, 5, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(16, 1, 3, 3, 3, 3, device=DEV)
    y = torch.empty(1, 4, 4, 5, 6, 16, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _ext.ext().conv1to16_kl(x, pack_kl_in(w), torch.zeros(16, device=DEV), None, y, 3, 1)
    h = torch.zeros(1, 4, 4, 5, 5, 16, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):   # 5x5 weights for a 3x3 launch
        _ext.ext().conv16to1_kl(h, pack_kl_out(torch.zeros(1, 16, 5, 5, 5, 5, device=DEV)), None,
                                torch.empty(1, 4, 4, 5, 5, device=DEV), 3, 1, 1.0)


# ---------------------------------------------------------------------------
# fused InLoc NC (csrc/nc_fused.hip)

def _nc_weights(seed):
    torch.manual_seed(seed)
    w1 = (torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.1).to(torch.bfloat16).float()
    b1 = 0.05 + torch.rand(16, device=DEV) * 0.1
    w2 = (torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.05).to(torch.bfloat16).float()
    b2 = torch.full((1,), 0.05, device=DEV)
    return w1, b1, w2, b2


@pytest.mark.parametrize("shape", [(2, 37, 50, 37, 50), (1, 9, 11, 13, 17), (2, 8, 7, 30, 41), (1, 3, 2, 5, 4)])
def test_nc_fused_k3_vs_oracle(shape):
    """relu(conv(relu(conv(x0, W1) + b1), W2) + b2) with the hidden layer rounded to bf16 like the kernel's LDS copy."""
    from ncnet_amd.ops.neigh_consensus import _fused_weights, _run_fused
    w1, b1, w2, b2 = _nc_weights(31)
    x0 = torch.rand(*shape, device=DEV).to(torch.bfloat16)
    wts = _fused_weights([ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)], [b1, b2])
    y = _run_fused(x0.contiguous(), wts)
    h = torch.relu(ref.conv4d(x0.double().unsqueeze(1), ref.conv4d_weight_from_std(w1.double()),
                              b1.double()))
    yr = torch.relu(ref.conv4d(bf(h), ref.conv4d_weight_from_std(w2.double()), b2.double()))[:, 0]
    assert not torch.isnan(y).any()
    assert rel_l2(y, yr) < 1e-2


def test_nc_fused_matches_layerwise_at_inloc_size(monkeypatch):
    """The symmetric NeighConsensus at the InLoc 3200 px volume (75x100x75x100): fused vs layer-by-layer HIP path."""
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    w1, b1, w2, b2 = _nc_weights(32)
    ws = [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)]
    x = torch.rand(1, 1, 75, 100, 75, 100, device=DEV)
    with torch.inference_mode():
        yf = nc.neigh_consensus(x, ws, [b1, b2], [16, 1])
        monkeypatch.setattr(nc, "FUSED", False)
        yl = nc.neigh_consensus(x, ws, [b1, b2], [16, 1])
    assert rel_l2(yf, yl) < 1e-2


def test_nc_fused_nonsquare_symmetric(monkeypatch):
    """(I, J) != (K, L): the swapped branch runs as its own launch."""
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    w1, b1, w2, b2 = _nc_weights(33)
    ws = [ref.conv4d_weight_from_std(w1), ref.conv4d_weight_from_std(w2)]
    x = torch.rand(1, 1, 6, 9, 11, 7, device=DEV)
    with torch.inference_mode():
        yf = nc.neigh_consensus(x, ws, [b1, b2], [16, 1])
    yr = ref.neigh_consensus(x.double(), [w.double() for w in ws], [b1.double(), b2.double()], True)
    assert rel_l2(yf, yr) < 1e-2
