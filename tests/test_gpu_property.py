"""Property-based GPU tests (Hypothesis): the HIP Conv4d
(forward, data- and weight-gradient through the autograd op) and the
correlation GEMM on random odd shapes, channel counts and kernel sizes vs the
fp64 oracles on bf16-rounded inputs.  Bounded: a handful of small examples
per test, derandomized, so a run stays within seconds on an MI355X."""
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
SET = settings(max_examples=8, deadline=None, derandomize=True, database=None)


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@SET
@given(cin=st.sampled_from([1, 3, 16, 17]), cout=st.sampled_from([1, 5, 16, 18]), ks=st.sampled_from([1, 3, 5, 7]),
       shape=st.tuples(st.integers(2, 9), st.integers(2, 9), st.integers(2, 30), st.integers(2, 30)),
       seed=st.integers(0, 2 ** 16))
def test_conv4d_random_shapes(cin, cout, ks, shape, seed):
    from ncnet_amd.ops.conv4d import conv4d
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.rand((2, cin) + shape, device=DEV, generator=g).to(torch.bfloat16).float().requires_grad_(True)
    w = (torch.randn(ks, cout, cin, ks, ks, ks, device=DEV, generator=g) * 0.05).to(torch.bfloat16).float()
    w.requires_grad_(True)
    b = (torch.randn(cout, device=DEV, generator=g) * 0.1).requires_grad_(True)
    before = _ext.DISPATCH["conv4d_hip"]
    y = conv4d(x, w, b, permute_filters=False)
    assert _ext.DISPATCH["conv4d_hip"] == before + 1
    gy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16).float()
    (y * gy).sum().backward()
    xr, wr, br = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = ref.conv4d(xr, wr, br)
    (yr * gy.double()).sum().backward()
    assert relerr(y, yr) < 1e-2
    assert relerr(x.grad, xr.grad) < 2e-2
    assert relerr(w.grad, wr.grad) < 2e-2
    assert relerr(b.grad, br.grad) < 1e-3


@SET
@given(m=st.integers(1, 700), n=st.integers(1, 700), k=st.sampled_from([64, 256, 1024]),
       batch=st.integers(1, 3), seed=st.integers(0, 2 ** 16))
def test_correlation_random_shapes(m, n, k, batch, seed):
    from ncnet_amd.ops.correlation import correlation
    g = torch.Generator(device=DEV).manual_seed(seed)
    a = torch.randn(batch, m, k, device=DEV, generator=g).to(torch.bfloat16).float()
    bb = torch.randn(batch, n, k, device=DEV, generator=g).to(torch.bfloat16).float()
    c = correlation(a, bb)
    cr = torch.bmm(a.double(), bb.double().transpose(1, 2))
    assert relerr(c, cr) < 1e-3
