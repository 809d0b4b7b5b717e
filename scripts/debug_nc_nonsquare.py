import torch
from ncnet_amd.ops import reference as ref
from ncnet_amd.ops.neigh_consensus import neigh_consensus
DEV = "cuda"
torch.manual_seed(4)
for shape in [(1, 1, 8, 10, 9, 7), (1, 1, 8, 10, 8, 10)]:
    x = torch.rand(shape, device=DEV).to(torch.bfloat16).float().requires_grad_(True)
    ws = [(torch.randn(3, 16, 1, 3, 3, 3, device=DEV) * 0.1).to(torch.bfloat16).float().requires_grad_(True),
          (torch.randn(3, 1, 16, 3, 3, 3, device=DEV) * 0.1).to(torch.bfloat16).float().requires_grad_(True)]
    bs = [(torch.rand(16, device=DEV) * 0.1).requires_grad_(True), (torch.rand(1, device=DEV) * 0.1).requires_grad_(True)]
    y = neigh_consensus(x, ws, bs, [16, 1], symmetric=True)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    xr = x.detach().double()
    wr = [w.detach().double().requires_grad_(True) for w in ws]
    br = [b.detach().double().requires_grad_(True) for b in bs]
    # oracle per branch
    def stack(v):
        h = torch.relu(ref.conv4d(v, wr[0], br[0]))
        pre = ref.conv4d(h, wr[1], br[1])
        return pre
    p1 = stack(xr)
    p2 = stack(ref.swap_ab(xr))
    g1 = g.double()
    g2 = ref.swap_ab(g.double())
    ob1 = float((g1 * (p1 > 0)).sum()); ob2 = float((g2 * (p2 > 0)).sum())
    print(shape, "hip gb1", float(bs[1].grad), "oracle", ob1 + ob2, "branch sums", ob1, ob2)
    print(" active frac", float((p1 > 0).double().mean()), float((p2 > 0).double().mean()),
          " |pre|<0.01 frac", float((p1.abs() < 1e-2).double().mean()))
    yr = torch.relu(p1) + ref.swap_ab(torch.relu(p2))
    print(" y relerr", float((y.double() - yr).norm() / yr.norm()))
