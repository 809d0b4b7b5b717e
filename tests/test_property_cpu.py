"""Property-based tests (Hypothesis, SURVEY.md section 4: random shapes and
odd sizes) of the oracles and of the NeighConsensus / Conv4d orchestration
on the exact CPU emulation of the HIP kernels (tests/emu_ext.py).

Examples are bounded (small volumes, fixed seeds per example, no deadline)
so the suite stays a few seconds on CPU."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.conv4d import Conv4dFn
from ncnet_amd.ops.neigh_consensus import NeighConsensusFn, layer_kinds
from tests.emu_ext import EmuExt

SET = settings(max_examples=12, deadline=None, derandomize=True,
               suppress_health_check=[HealthCheck.function_scoped_fixture])
dims = st.integers(min_value=2, max_value=6)


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture
def emu(monkeypatch):
    monkeypatch.setattr(_ext, "_C", EmuExt)
    monkeypatch.setattr(_ext, "load", lambda: EmuExt)
    yield


def brute_conv4d(x, w_std, b):
    """Direct 4D cross-correlation with zero 'same' padding (the definition)."""
    V, ci, I, J, K, L = x.shape
    co, _, k = w_std.shape[0], w_std.shape[1], w_std.shape[2]
    p = k // 2
    xp = torch.nn.functional.pad(x, (p, p, p, p, p, p, p, p))
    y = torch.zeros(V, co, I, J, K, L, dtype=x.dtype)
    for a in range(k):
        for bb in range(k):
            for c in range(k):
                for d in range(k):
                    patch = xp[:, :, a:a + I, bb:bb + J, c:c + K, d:d + L]
                    y += torch.einsum("vcijkl,oc->voijkl", patch, w_std[:, :, a, bb, c, d])
    return y + b.view(1, -1, 1, 1, 1, 1)


@SET
@given(I=dims, J=dims, K=dims, L=dims, ks=st.sampled_from([1, 3, 5]), cin=st.integers(1, 3),
       cout=st.integers(1, 3), seed=st.integers(0, 2 ** 16))
def test_conv4d_oracle_is_the_definition(I, J, K, L, ks, cin, cout, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(2, cin, I, J, K, L, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, ks, ks, ks, ks, generator=g, dtype=torch.float64)
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    y = ref.conv4d(x, ref.conv4d_weight_from_std(w), b)
    assert torch.allclose(y, brute_conv4d(x, w, b), atol=1e-9)


@SET
@given(I=dims, J=dims, K=dims, L=dims, seed=st.integers(0, 2 ** 16))
def test_mutual_matching_commutes_with_swap(I, J, K, L, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(2, 1, I, J, K, L, generator=g, dtype=torch.float64)
    a = ref.swap_ab(ref.mutual_matching(x))
    b = ref.mutual_matching(ref.swap_ab(x))
    assert torch.allclose(a, b)
    # and it never increases a value (both ratios are <= 1 on non-negative volumes)
    assert (ref.mutual_matching(x) <= x + 1e-12).all()


@SET
@given(i=st.integers(1, 4), j=st.integers(1, 4), k=st.integers(1, 4), l=st.integers(1, 4),
       ks=st.sampled_from([2, 3]), seed=st.integers(0, 2 ** 16))
def test_maxpool4d_values_and_offsets(i, j, k, l, ks, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(3, 1, i * ks, j * ks, k * ks, l * ks, generator=g)
    val, off = ref.maxpool4d(x, ks)
    assert val.shape == (3, 1, i, j, k, l)
    di, dj, dk, dl = (o.long() for o in off)
    # the offsets address the maximum of each window, per batch element
    I = torch.arange(i).view(1, 1, -1, 1, 1, 1) * ks + di
    J = torch.arange(j).view(1, 1, 1, -1, 1, 1) * ks + dj
    K = torch.arange(k).view(1, 1, 1, 1, -1, 1) * ks + dk
    L = torch.arange(l).view(1, 1, 1, 1, 1, -1) * ks + dl
    v = torch.arange(3).view(-1, 1, 1, 1, 1, 1)
    picked = x[v, 0, I, J, K, L].reshape(val.shape)
    assert torch.equal(picked, val)


@SET
@given(I=dims, J=dims, seed=st.integers(0, 2 ** 16), norm=st.sampled_from(["softmax", "l1", None]))
def test_weak_loss_score_closed_forms(I, J, seed, norm):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(2, 1, I, J, I, J, generator=g, dtype=torch.float64) * 3
    s = ref.match_score(x, norm)
    B = x.view(2, I * J, I * J)
    if norm == "softmax":      # max of a softmax = 1 / sum exp(x - max)   (train.py:121-134)
        sb = 1.0 / torch.exp(B - B.max(1, keepdim=True).values).sum(1)
        sa = 1.0 / torch.exp(B - B.max(2, keepdim=True).values).sum(2)
    elif norm == "l1":
        sb = (B / (B.sum(1, keepdim=True) + ref.L1_EPS)).max(1).values
        sa = (B / (B.sum(2, keepdim=True) + ref.L1_EPS)).max(2).values
    else:
        sb, sa = B.max(1).values, B.max(2).values
    assert torch.allclose(s, (sa + sb).mean() / 2, rtol=1e-9)


STACKS = st.sampled_from([((3, 3), (16, 1)), ((3,), (1,)), ((3, 3), (5, 1)), ((1, 3), (16, 1)),
                          ((3, 3), (18, 1)), ((3, 3), (4, 20))])


@SET
@given(stack=STACKS, I=st.integers(2, 5), J=st.integers(2, 5), K=st.integers(2, 5), L=st.integers(2, 5),
       symmetric=st.booleans(), seed=st.integers(0, 2 ** 16))
def test_nc_orchestration_random_shapes(emu, stack, I, J, K, L, symmetric, seed):
    """NeighConsensusFn (channel blocks, ij encodings, symmetric batching,
    backward routing) on the kernel emulator vs autograd of the fp64 oracle,
    positive weights so bf16 storage stays < 1 % and any routing error shows."""
    ks, ch = stack
    g = torch.Generator().manual_seed(seed)
    ws, bs, cin = [], [], 1
    for k, c in zip(ks, ch):
        w = (torch.rand(c, cin, k, k, k, k, generator=g) + 0.1) * (1.0 / (cin * k ** 4))
        ws.append(ref.conv4d_weight_from_std(w).requires_grad_(True))
        bs.append((torch.rand(c, generator=g) * 0.1).requires_grad_(True))
        cin = c
    kinds = layer_kinds(list(ch), list(ks))
    x = torch.rand(2, 1, I, J, K, L, generator=g).to(torch.bfloat16).float()
    xa = x.clone().requires_grad_(True)
    params = [t for pair in zip(ws, bs) for t in pair]
    y = NeighConsensusFn.apply(xa, symmetric, tuple(kinds), tuple(ch), *params)
    gy = torch.rand(y.shape, generator=g)
    (y * gy).sum().backward()
    xr = x.double().requires_grad_(True)
    wd = [w.detach().double().requires_grad_(True) for w in ws]
    bd = [b.detach().double().requires_grad_(True) for b in bs]
    yr = ref.neigh_consensus(xr, wd, bd, symmetric)
    (yr * gy.double()).sum().backward()
    errs = [rl2(y, yr), rl2(xa.grad, xr.grad)] + [rl2(p.grad, q.grad) for p, q in
                                                   zip(params, [t for pair in zip(wd, bd) for t in pair])]
    assert max(errs) < 1.5e-2, errs


@SET
@given(cin=st.integers(1, 20), cout=st.integers(1, 20), ks=st.sampled_from([1, 3, 5]),
       shape=st.tuples(st.integers(2, 4), st.integers(2, 4), st.integers(2, 4), st.integers(2, 4)),
       seed=st.integers(0, 2 ** 16))
def test_conv4d_module_random_channels(emu, cin, cout, ks, shape, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((1, cin) + shape, generator=g).to(torch.bfloat16).float()
    w = ref.conv4d_weight_from_std((torch.rand(cout, cin, ks, ks, ks, ks, generator=g) + 0.1) * 0.1)
    w.requires_grad_(True)
    b = (torch.rand(cout, generator=g) * 0.1).requires_grad_(True)
    xa = x.clone().requires_grad_(True)
    y = Conv4dFn.apply(xa, w, b)
    gy = torch.rand(y.shape, generator=g)
    (y * gy).sum().backward()
    xr = x.double().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    br = b.detach().double().requires_grad_(True)
    yr = ref.conv4d(xr, wr, br)
    (yr * gy.double()).sum().backward()
    errs = [rl2(y, yr), rl2(xa.grad, xr.grad), rl2(w.grad, wr.grad), rl2(b.grad, br.grad)]
    assert max(errs) < 1.5e-2, errs
