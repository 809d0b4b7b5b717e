"""Per-GPU batches past the int32 index range (BASELINE config 2: batch sized
for 288 GB of HBM).  At 400 px and per-GPU batch 48 the ij-packed layer-1
input holds 2 groups x 192 volumes x 25^4 voxels x 16 channels = 2.4e9
elements and the layer-3 fp32 partials 25 x 7.5e7 = 1.9e9: every kernel
index must be 64-bit.  The fused training path at batch 48 must reproduce,
pair for pair, three independent batch-16 runs on the same features
(positives only: the rolled negatives wrap at the batch boundary)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_batch48_matches_batch16_chunks():
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(DEV)
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.05)
    m.train()
    B, b = 48, 16
    g = torch.Generator(device=DEV).manual_seed(3)
    src = torch.randn(B, 3, 400, 400, device=DEV, generator=g)
    tgt = torch.randn(B, 3, 400, 400, device=DEV, generator=g)
    with torch.no_grad():
        f, hw = m.extract(torch.cat((src, tgt)))
    fs, ft = f[:B], f[B:]
    params = list(m.NeighConsensus.parameters())

    def run(fa, fb):
        n = fa.shape[0]
        vols = m.weak_loss_volumes_from_features(torch.cat((fa, fb)), hw, n)
        gsel = torch.zeros_like(vols)
        gsel[:n] = torch.linspace(-1, 1, vols[:n].numel(), device=DEV).view_as(vols[:n])
        grads = torch.autograd.grad((vols * gsel).sum(), params)
        return vols[:n].detach(), grads

    big_v, big_g = run(fs, ft)
    assert torch.isfinite(big_v).all()
    acc = None
    gs_all = torch.linspace(-1, 1, big_v.numel(), device=DEV).view_as(big_v)
    for c in range(B // b):
        sl = slice(c * b, (c + 1) * b)
        vols = m.weak_loss_volumes_from_features(torch.cat((fs[sl], ft[sl])), hw, b)
        # the chunk's positives equal the big batch's (per-volume ops only)
        d = float((vols[:b].detach() - big_v[sl]).abs().max())
        assert d == 0.0, d
        # gradients: the chunk weighted by its slice of the big run's upstream gradient
        gsel = torch.zeros_like(vols)
        gsel[:b] = gs_all[sl]
        gr = torch.autograd.grad((vols * gsel).sum(), params)
        acc = list(gr) if acc is None else [a + x for a, x in zip(acc, gr)]
    for a, x in zip(acc, big_g):
        rel = float((a - x).norm() / x.norm().clamp_min(1e-30))
        assert rel < 2e-3, rel
