"""Stage-by-stage check of the fused NeighConsensus backward against a
*quantized* fp64 oracle that rounds to bf16 at exactly the points where the
HIP path stores bf16 (layer activations, layer gradients, packed weights).
Any difference left is fp32-vs-fp64 accumulation order, so tolerances are
tight and a mismatch localises a bug to one stage."""
import pytest
import torch

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.neigh_consensus import _stack_bwd, _stack_fwd, blocks_to_ncl, layer_kinds, planar_to_blocks

pytestmark = pytest.mark.gpu
DEV = "cuda"


def q(x):
    return x.to(torch.bfloat16).double()


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def conv_fwd(x, w_std):  # x [V,C,I,J,K,L] fp64
    return ref.conv4d(x, ref.conv4d_weight_from_std(w_std))


def grads(x, w_std, g):
    x = x.detach().requires_grad_(True)
    w = w_std.detach().requires_grad_(True)
    (conv_fwd(x, w) * g).sum().backward()
    return x.grad, w.grad


@pytest.mark.parametrize("ks,ch", [((5, 5, 5), (16, 16, 1)), ((3, 3), (16, 1)), ((3, 3, 3), (10, 10, 1)),
                                   ((5, 5), (32, 1)), ((7, 3), (16, 1)), ((1, 3), (16, 1)), ((3, 3), (20, 24))])
def test_stack_stages_vs_quantized_oracle(ks, ch):
    torch.manual_seed(11)
    V, I, J, K, L = 3, 9, 8, 10, 11
    x0 = torch.rand(V, I, J, K, L, device=DEV).to(torch.bfloat16)
    ws_ref, bs, ws_std = [], [], []
    cin = 1
    for k, c in zip(ks, ch):
        w_std = q(torch.randn(c, cin, k, k, k, k, device=DEV) * 0.1)
        ws_std.append(w_std)
        ws_ref.append(ref.conv4d_weight_from_std(w_std).float())
        bs.append(torch.rand(c, device=DEV) * 0.1)
        cin = c
    kinds = layer_kinds(list(ch), list(ks))
    saved = []
    z = _stack_fwd(x0.contiguous(), ws_ref, bs, kinds, saved)
    # quantized oracle forward
    hs = [x0.double().unsqueeze(1)]
    for li, (w, b) in enumerate(zip(ws_std, bs)):
        pre = conv_fwd(hs[-1], w) + b.double().view(1, -1, 1, 1, 1, 1)
        act = torch.relu(pre)
        hs.append(act if li == len(ks) - 1 else q(act))
    zl = z.unsqueeze(1) if ch[-1] == 1 else z.transpose(0, 1)      # [V, C, I, J, K, L]
    errs = {"z": rl2(zl, hs[-1])}
    for li in range(1, len(ks)):
        errs[f"h{li}"] = rl2(blocks_to_ncl(saved[li], ch[li - 1]), hs[li])
    # backward from a random gradient on z
    gz = torch.randn_like(zl)
    gm = gz * (zl > 0)
    g_last = gm[:, 0].to(torch.bfloat16) if ch[-1] == 1 else planar_to_blocks(gm.transpose(0, 1))
    dws, dbs, gx0 = _stack_bwd(g_last, saved, ws_ref, kinds, list(ch), True)
    g = q(gz.double() * (hs[-1] > 0))
    for li in range(len(ks) - 1, -1, -1):
        gx, gw = grads(hs[li], ws_std[li], g)
        errs[f"dw{li}"] = rl2(ref.conv4d_weight_to_std(dws[li]), gw)
        errs[f"db{li}"] = rl2(dbs[li], g.sum(dim=(0, 2, 3, 4, 5)))
        if li > 0:
            g = q(gx * (hs[li] > 0))
        else:
            errs["gx0"] = rl2(gx0, gx[:, 0])
    assert max(errs.values()) < 5e-3, errs


@pytest.mark.parametrize("shape", [(2, 1, 6, 7, 6, 7), (1, 1, 8, 10, 9, 7)])
def test_symmetric_vs_nonsymmetric_consistency(shape):
    """symmetric NC == stack(x) + swap(stack(swap(x))) computed with two
    non-symmetric calls of the same HIP op (forward and all gradients)."""
    from ncnet_amd.ops.neigh_consensus import neigh_consensus
    torch.manual_seed(12)
    x = torch.rand(shape, device=DEV).to(torch.bfloat16).float()
    ws = [(torch.randn(3, 16, 1, 3, 3, 3, device=DEV) * 0.1).requires_grad_(True),
          (torch.randn(3, 1, 16, 3, 3, 3, device=DEV) * 0.1).requires_grad_(True)]
    bs = [(torch.rand(16, device=DEV) * 0.1).requires_grad_(True), (torch.rand(1, device=DEV) * 0.1).requires_grad_(True)]
    xa = x.clone().requires_grad_(True)
    y = neigh_consensus(xa, ws, bs, [16, 1], symmetric=True)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    gs = [w.grad.clone() for w in ws] + [b.grad.clone() for b in bs] + [xa.grad.clone()]
    for t in ws + bs:
        t.grad = None
    xb = x.clone().requires_grad_(True)
    y1 = neigh_consensus(xb, ws, bs, [16, 1], symmetric=False)
    y2 = ref.swap_ab(neigh_consensus(ref.swap_ab(xb).contiguous(), ws, bs, [16, 1], symmetric=False))
    ys = y1 + y2
    (ys * g).sum().backward()
    gn = [w.grad.clone() for w in ws] + [b.grad.clone() for b in bs] + [xb.grad.clone()]
    errs = {"y": rl2(y, ys)}
    errs.update({f"g{i}": rl2(a, b) for i, (a, b) in enumerate(zip(gs, gn))})
    assert max(errs.values()) < 1e-4, errs


def test_combine_nonsquare():
    torch.manual_seed(13)
    V, R, C = 2, 80, 63
    z = torch.randn(2 * V * R * C, device=DEV)
    y = torch.empty(V, R, C, device=DEV)
    _ext.ext().combine_fwd(z, y, R, C)
    z1, z2 = z[:V * R * C].view(V, R, C), z[V * R * C:].view(V, C, R)
    assert torch.allclose(y, z1 + z2.transpose(1, 2))
    g = torch.randn(V, R, C, device=DEV)
    gz = torch.empty(2 * V * R * C, device=DEV, dtype=torch.bfloat16)
    _ext.ext().combine_bwd(g, z, gz, R, C)
    e1 = (g * (z1 > 0)).to(torch.bfloat16)
    e2 = (g.transpose(1, 2) * (z2 > 0)).to(torch.bfloat16)
    assert torch.equal(gz[:V * R * C].view(V, R, C), e1)
    assert torch.equal(gz[V * R * C:].view(V, C, R), e2)
