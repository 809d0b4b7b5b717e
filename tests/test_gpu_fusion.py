"""Round-5 launch fusions of the training step, each against the unfused path
it replaces (bit for bit where the arithmetic is the same):

* MutualMatching writing the padded NC-input planes of both symmetric branches
  (mm_apply PAD mode, halos included) == zero fill + the two pad_planes passes;
* the one-launch weight packs (packing.packed_weights) == the per-pack packers;
* the weak-loss score sum (score_sum) and the in-kernel gradient scale of
  softmax_max_bwd == the PyTorch forms;
* ImMatchNet.process_correlation with the padded MutualMatching == separate
  MutualMatching + NeighConsensus (forward and every gradient, bit for bit).
"""
import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import packing as P
from ncnet_amd.ops.reference import conv4d_weight_to_std

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("ks,n", [(5, 25), (5, 20), (3, 25), (5, 7)])
def test_mm_apply_padded_planes_equal_pad_passes(ks, n):
    torch.manual_seed(ks * 100 + n)
    C = _ext.ext()
    V, R = 3, n * n
    c3 = torch.rand(V, R, R, device=DEV)
    rmax, cmax = c3.amax(2).contiguous(), c3.amax(1).contiguous()
    out = torch.empty_like(c3)
    C.mm_apply(c3, rmax, cmax, out, None, None, 1e-5)
    _, ppl = C.pad_geom(n, n, ks)
    want = torch.zeros((2 * V * R, ppl), dtype=torch.bfloat16, device=DEV)
    C.pad_planes(out, want[:V * R], n, n, ks, 0)
    C.pad_planes(out, want[V * R:], n, n, ks, 1)
    got = torch.full((2 * V * R, ppl), float("nan"), dtype=torch.bfloat16, device=DEV)   # halos must be written
    out2 = torch.empty_like(c3)
    C.mm_apply(c3, rmax, cmax, out2, got[:V * R], got[V * R:], 1e-5, [ks, n, n])
    assert torch.equal(out2, out)
    assert torch.equal(got, want)


@pytest.mark.parametrize("ks", [3, 5])
def test_packed_weights_gpu_equal_packers(ks):
    torch.manual_seed(ks)
    flat = torch.randn(250000, device=DEV)
    shapes = [(ks, 16, 1, ks, ks, ks), (ks, 16, 16, ks, ks, ks), (ks, 1, 16, ks, ks, ks)]
    ws, o = [], 11
    for sh in shapes:
        n = int(torch.tensor(sh).prod())
        ws.append(flat[o:o + n].view(sh))
        o += n + 5
    specs = [(0, P.pack_w1x), (1, P.pack_w16), (1, P._w16_dgrad), (2, P._blk_packed), (2, P._w1x_dgrad)]
    for shared in (True, False):
        src = ws if shared else [w.clone() for w in ws]
        got = P.packed_weights(src, specs)
        for (wi, fn), g in zip(specs, got):
            want = fn(conv4d_weight_to_std(src[wi]).float()).to(torch.bfloat16)
            assert torch.equal(g, want), (shared, fn.__name__)
    # an in-place update (version bump) re-packs; an unchanged weight reuses the packs
    a = P.packed_weights(ws, specs)
    assert P.packed_weights(ws, specs)[0] is a[0]
    with torch.no_grad():
        ws[0].mul_(2.0)
    b = P.packed_weights(ws, specs)
    assert b[0] is not a[0]
    assert torch.equal(b[0], P.pack_w1x(conv4d_weight_to_std(ws[0]).float()).to(torch.bfloat16))


def test_pack_cache_keyed_on_weight_objects():
    """A model freed and a new one of the same shape (whose weights the
    caching allocator may place at the old addresses, with equal version
    counters) must never get the old model's packs; a ``p.data`` edit (no
    version bump) re-packs after clear_pack_cache (ImMatchNet.load_state_dict)."""
    ks = 5
    shapes = [(ks, 16, 1, ks, ks, ks), (ks, 16, 16, ks, ks, ks), (ks, 1, 16, ks, ks, ks)]
    specs = [(0, P.pack_w1x), (1, P.pack_w16), (2, P._blk_packed)]

    def model(seed):
        g = torch.Generator(device=DEV).manual_seed(seed)
        return [torch.nn.Parameter(torch.randn(sh, device=DEV, generator=g)) for sh in shapes]

    for seed in range(4):
        ws = model(seed)
        got = [g.clone() for g in P.packed_weights(ws, specs)]
        for (wi, fn), g in zip(specs, got):
            assert torch.equal(g, fn(conv4d_weight_to_std(ws[wi]).float()).to(torch.bfloat16)), seed
        del ws
    ws = model(7)
    a = P.packed_weights(ws, specs)
    ws[1].data.mul_(3.0)                     # no version bump
    P.clear_pack_cache()
    b = P.packed_weights(ws, specs)
    assert torch.equal(b[1], P.pack_w16(conv4d_weight_to_std(ws[1]).float()).to(torch.bfloat16))
    assert not torch.equal(a[1], b[1])


@pytest.mark.parametrize("norm", [0, 1, 2])
def test_score_sum_and_gscale(norm):
    from ncnet_amd.ops import loss as L
    torch.manual_seed(norm)
    x = torch.rand(4, 49, 36, device=DEV)
    wr, wc = torch.randn(4, device=DEV), torch.randn(4, device=DEV)
    st = L._row_col_stats(x, norm)
    rmax, rarg, rse, cmax, carg, cse = st
    val = torch.empty((), device=DEV)
    _ext.ext().score_sum(rmax, rse, cmax, cse, wr, wc, val, norm, 1e-4)

    def sc(mx, s):
        return 1.0 / s if norm == 1 else mx / (s + 1e-4) if norm == 2 else mx
    want = (wr.view(-1, 1) * sc(rmax, rse)).sum() + (wc.view(-1, 1) * sc(cmax, cse)).sum()
    assert abs(float(val) - float(want)) <= 1e-5 * max(1.0, abs(float(want)))
    g0, g1 = torch.empty_like(x), torch.empty_like(x)
    gs = torch.tensor([0.37], device=DEV)
    _ext.ext().softmax_max_bwd(x, rmax, rarg, rse, cmax, carg, cse, wr, wc, g0, norm, 1e-4)
    _ext.ext().softmax_max_bwd(x, rmax, rarg, rse, cmax, carg, cse, wr, wc, g1, norm, 1e-4, gs)
    assert torch.equal(g1, g0 * gs)


def test_process_correlation_padded_mm_bitwise():
    """The training step's MutualMatching -> NeighConsensus with the planes
    written by MutualMatching vs the un-fused path: identical outputs and
    gradients (the same kernels read the same bf16 planes)."""
    from ncnet_amd.models.immatchnet import MutualMatching, NeighConsensus
    torch.manual_seed(7)
    nc = NeighConsensus(kernel_sizes=[5, 5, 5], channels=[16, 16, 1]).to(DEV)
    corr = torch.rand(4, 1, 25, 25, 25, 25, device=DEV)
    g = torch.randn(4, 1, 25, 25, 25, 25, device=DEV)
    res = []
    for fused in (False, True):
        c = corr.clone().requires_grad_(True)
        nc.zero_grad(set_to_none=True)
        ks = nc.padded_input_ks(c)
        assert ks == 5
        if fused:
            from ncnet_amd.ops.mutual import mutual_matching_padded
            x, xp = mutual_matching_padded(c, ks)
            y = nc(x, padded=xp)
        else:
            y = nc(MutualMatching(c))
        (y * g).sum().backward()
        res.append([y.detach().clone(), c.grad.clone()] + [p.grad.clone() for p in nc.parameters()])
    names = ["y", "d corr"] + [n for n, _ in nc.named_parameters()]
    for name, a, b in zip(names, *res):
        if name in ("y", "d corr"):
            assert torch.equal(a, b), name
        else:
            # weight gradients: the 1-channel wgrad kernels merge their wave
            # partials with LDS float atomics (order not fixed): within fp32 rounding
            err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
            assert err < 1e-5, (name, err)


def test_reduce_cols_matches_torch_layouts():
    """reduce_cols (one launch for up to four segments: column sums of the
    weight-gradient partials scattered into the checkpoint layout) against the
    torch path of reduce_partials; the fixed summation order makes two runs
    bitwise equal."""
    import importlib
    from ncnet_amd.ops import reference as ref
    nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")
    torch.manual_seed(1)
    ks = 5
    p16 = torch.randn(204, ks * ks, ks * ks, 16, 16, device=DEV)
    pb = torch.randn(204, 16, device=DEV)
    p1x = torch.randn(256, ks * ks, 32, 16, device=DEV)
    f16 = lambda t: ref.conv4d_weight_from_std(nc._reduce_wgrad16(t, ks, 16, 16))  # noqa: E731
    f_last = lambda t: t[:, :25, :16].reshape((ks,) * 4 + (16,)).flip(0, 1, 2, 3).permute(2, 4, 3, 0, 1).unsqueeze(1)  # noqa: E731
    segs = [(p16, ("g16", ks), f16), (pb, None, None), (p1x, ("gl", ks), f_last)]
    got = nc.reduce_partials(segs)
    again = nc.reduce_partials(segs)
    want = [f16(p16.double().sum(0)), pb.double().sum(0), f_last(p1x.double().sum(0))]
    for g, a, w in zip(got, again, want):
        assert g.shape == w.shape
        assert torch.equal(g, a)
        assert torch.allclose(g.double(), w, rtol=1e-5, atol=1e-4), (g.double() - w).abs().max()
