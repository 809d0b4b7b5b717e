"""The one-launch weight packing (ops/packing.py packed_weights): the index plan
of every pack, applied as a plain gather on the CPU, reproduces the per-pack
PyTorch packers exactly -- both from a concatenated source and from one shared
flat storage (FlatAdam's), at the training stack's kinds and kernel sizes."""
import pytest
import torch

from ncnet_amd.ops import packing as P
from ncnet_amd.ops.reference import conv4d_weight_to_std


def _emulate(ws, specs, shared: bool):
    if shared:
        flat = torch.cat([w.reshape(-1) for w in ws] + [torch.randn(7)])
        views, o = [], 3
        flat = torch.cat((torch.randn(3), flat))
        for w in ws:
            views.append(flat[o:o + w.numel()].view(w.shape))
            o += w.numel()
        src = P._source(views)
        assert src is not None
        flat, offs = src
        ws = views
    else:
        assert P._source(ws) is None
        flat = torch.cat([w.reshape(-1) for w in ws])
        offs, o = [], 0
        for w in ws:
            offs.append(o)
            o += w.numel()
    idx, shp = P._plan(tuple(tuple(w.shape) for w in ws), offs, flat.numel(), tuple(specs), "cpu")
    vals = torch.where(idx >= 0, flat[idx.clamp(min=0).long()], torch.zeros(()))
    outs, o = [], 0
    for sh in shp:
        n = int(torch.tensor(sh).prod())
        outs.append(vals[o:o + n].view(sh))
        o += n
    return ws, outs


@pytest.mark.parametrize("ks", [3, 5])
@pytest.mark.parametrize("shared", [False, True])
def test_packed_weights_plan_matches_packers(ks, shared):
    torch.manual_seed(ks)
    ws = [torch.randn(ks, 16, 1, ks, ks, ks), torch.randn(ks, 16, 16, ks, ks, ks), torch.randn(ks, 1, 16, ks, ks, ks)]
    specs = [(0, P.pack_w1x), (1, P.pack_w16), (1, P._w16_dgrad), (2, P._blk_packed), (2, P._w1x_dgrad)]
    ws, outs = _emulate(ws, specs, shared)
    for (wi, fn), got in zip(specs, outs):
        want = fn(conv4d_weight_to_std(ws[wi]).float())
        assert got.shape == want.shape
        assert torch.equal(got.to(torch.bfloat16), want.to(torch.bfloat16)), fn.__name__


def test_reduce_partials_layouts_cpu():
    """ops/neigh_consensus.reduce_partials (the CPU path of the reduce_cols
    launch): the scatter map built from the layout function reproduces
    layout(part.sum(0)) for the three weight-gradient layouts of the training
    stack, slices included."""
    from ncnet_amd.ops import reference as ref
    from ncnet_amd.ops.neigh_consensus import _reduce_wgrad16, reduce_partials
    torch.manual_seed(0)
    ks = 5
    p16 = torch.randn(6, ks * ks, ks * ks, 16, 16)
    pb = torch.randn(6, 16)
    p1x = torch.randn(5, ks * ks, 32, 16)
    f16 = lambda t: ref.conv4d_weight_from_std(_reduce_wgrad16(t, ks, 16, 16))  # noqa: E731
    f_first = lambda t: t[:, :25, :16].reshape((ks,) * 4 + (16,)).permute(2, 4, 3, 0, 1).unsqueeze(2)  # noqa: E731
    f_last = lambda t: t[:, :25, :7].reshape((ks,) * 4 + (7,)).flip(0, 1, 2, 3).permute(2, 4, 3, 0, 1).unsqueeze(1)  # noqa: E731
    got = reduce_partials([(p16, ("t16", ks), f16), (pb, None, None), (p1x, ("tf", ks), f_first),
                           (p1x, ("tl", ks, 7), f_last)])
    want = [f16(p16.sum(0)), pb.sum(0), f_first(p1x.sum(0)), f_last(p1x.sum(0))]
    for g, w in zip(got, want):
        assert g.shape == w.shape
        assert torch.allclose(g, w, rtol=1e-6, atol=1e-6)
