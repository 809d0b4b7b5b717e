"""CPU tests of the oracles, the model plumbing (BASELINE config 0) and the
reference-compatibility contracts (checkpoint layout, CLI semantics)."""
import argparse
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

from ncnet_amd.ops import reference as ref


def test_conv4d_oracle_matches_bruteforce():
    torch.manual_seed(0)
    x = torch.randn(2, 3, 5, 4, 6, 5, dtype=torch.float64)
    w_std = torch.randn(4, 3, 3, 3, 3, 3, dtype=torch.float64)
    b = torch.randn(4, dtype=torch.float64)
    y = ref.conv4d(x, ref.conv4d_weight_from_std(w_std), b)
    xp = torch.nn.functional.pad(x, (1, 1, 1, 1, 1, 1, 1, 1))
    yb = torch.zeros_like(y)
    for a in range(3):
        for c in range(3):
            for d in range(3):
                for e in range(3):
                    sl = xp[:, :, a:a + 5, c:c + 4, d:d + 6, e:e + 5]
                    yb += torch.einsum("nijklm,oi->nojklm", sl, w_std[:, :, a, c, d, e])
    yb += b.view(1, -1, 1, 1, 1, 1)
    assert torch.allclose(y, yb, atol=1e-10)
    # the reference slice-loop algorithm agrees too
    ys = ref.conv4d_sliced(x, ref.conv4d_weight_from_std(w_std), b)
    assert torch.allclose(ys, yb, atol=1e-10)


def test_mutual_matching_symmetry_and_formula():
    torch.manual_seed(1)
    c = torch.rand(2, 1, 4, 5, 4, 5, dtype=torch.float64)
    out = ref.mutual_matching(c)
    out_t = ref.swap_ab(ref.mutual_matching(ref.swap_ab(c)))
    assert torch.equal(out, out_t)
    m = c.reshape(2, 20, 20)
    ra = m.max(2, keepdim=True)[0] + 1e-5
    cb = m.max(1, keepdim=True)[0] + 1e-5
    assert torch.allclose(out.reshape(2, 20, 20), m * (m / ra) * (m / cb))


def test_maxpool4d_batch_correct_int_offsets():
    torch.manual_seed(2)
    c = torch.rand(3, 1, 4, 6, 4, 2)
    v, (di, dj, dk, dl) = ref.maxpool4d(c, 2)
    assert v.shape == (3, 1, 2, 3, 2, 1) and di.dtype == torch.int64
    for b in range(3):
        for i in range(2):
            for j in range(3):
                for k in range(2):
                    blk = c[b, 0, 2 * i:2 * i + 2, 2 * j:2 * j + 2, 2 * k:2 * k + 2, 0:2]
                    assert v[b, 0, i, j, k, 0] == blk.max()
                    o = (di[b, 0, i, j, k, 0], dj[b, 0, i, j, k, 0], dk[b, 0, i, j, k, 0], dl[b, 0, i, j, k, 0])
                    assert blk[o] == blk.max()


def test_softmax_max_closed_form():
    torch.manual_seed(3)
    x = torch.randn(2, 1, 3, 4, 3, 4, dtype=torch.float64)
    sa, sb = ref.softmax_max_scores(x)
    m = x.reshape(2, 12, 12)
    assert torch.allclose(sb, 1 / torch.exp(m - m.max(1, keepdim=True)[0]).sum(1))
    assert torch.allclose(sa, 1 / torch.exp(m - m.max(2, keepdim=True)[0]).sum(2))


def test_immatchnet_config0_cpu_forward():
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    batch = {"source_image": torch.randn(1, 3, 200, 200), "target_image": torch.randn(1, 3, 200, 200)}
    with torch.no_grad():
        out = m(batch)
    assert out.shape == (1, 1, 13, 13, 13, 13)
    assert torch.isfinite(out).all() and (out >= 0).all()


def test_relocalization_forward_cpu():
    from ncnet_amd.models import ImMatchNet
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False, relocalization_k_size=2)
    batch = {"source_image": torch.randn(1, 3, 192, 256), "target_image": torch.randn(1, 3, 192, 256)}
    with torch.no_grad():
        out, delta = m(batch)
    assert out.shape == (1, 1, 6, 8, 6, 8) and len(delta) == 4
    assert all(d.shape == out.shape and d.max() <= 1 and d.min() >= 0 for d in delta)
    # eval_inloc.py's query-feature reuse: extract once, match per pano == forward of the pair
    with torch.no_grad():
        fq, fp = m.extract(batch["source_image"]), m.extract(batch["target_image"])
        out2, delta2 = m.match_features(fq[0], fq[1], fp[0], fp[1])
    assert torch.equal(out, out2) and all(torch.equal(a, b) for a, b in zip(delta, delta2))


def test_state_dict_keys_match_reference_layout():
    from ncnet_amd.models import ImMatchNet
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], use_cuda=False)
    sd = m.state_dict()
    assert sd["NeighConsensus.conv.0.weight"].shape == (5, 16, 1, 5, 5, 5)
    assert sd["NeighConsensus.conv.2.weight"].shape == (5, 16, 16, 5, 5, 5)
    assert sd["NeighConsensus.conv.4.weight"].shape == (5, 1, 16, 5, 5, 5)
    assert sd["FeatureExtraction.model.0.weight"].shape == (64, 3, 7, 7)
    assert "FeatureExtraction.model.6.22.conv3.weight" in sd  # layer3 has 23 blocks
    assert "FeatureExtraction.model.4.0.downsample.1.running_var" in sd
    n_nc = sum(p.numel() for p in m.NeighConsensus.parameters())
    assert n_nc == 180033


def _fake_reference_checkpoint(path, ks=(3, 3), ch=(16, 1), legacy_vgg=False):
    """A checkpoint laid out like train.py:197-205 writes it."""
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(5)
    m = ImMatchNet(ncons_kernel_sizes=list(ks), ncons_channels=list(ch), use_cuda=False)
    sd = OrderedDict((k, v.clone()) for k, v in m.state_dict().items() if "num_batches_tracked" not in k)
    if legacy_vgg:
        sd = OrderedDict((k.replace("model", "vgg") if k.startswith("FeatureExtraction") else k, v) for k, v in sd.items())
    args = argparse.Namespace(checkpoint="", image_size=400, dataset_image_path="x", dataset_csv_path="y",
                              num_epochs=5, batch_size=16, lr=0.0005, ncons_kernel_sizes=list(ks),
                              ncons_channels=list(ch), result_model_fn="checkpoint_adam",
                              result_model_dir="trained_models", fe_finetune_params=0)
    state = {"epoch": 3, "args": args, "state_dict": sd, "best_test_loss": 0.1,
             "optimizer": torch.optim.Adam(m.NeighConsensus.parameters()).state_dict(),
             "train_loss": np.zeros(5), "test_loss": np.array([0.3, 0.2, 0.1, 0.0, 0.0])}
    torch.save(state, path)
    return m


@pytest.mark.parametrize("legacy_vgg", [False, True])
def test_load_reference_layout_checkpoint(tmp_path, legacy_vgg):
    from ncnet_amd.models import ImMatchNet
    p = str(tmp_path / "ncnet.pth.tar")
    src = _fake_reference_checkpoint(p, legacy_vgg=legacy_vgg)
    # constructor kwargs are overridden by checkpoint args (lib/model.py:217-219)
    m = ImMatchNet(checkpoint=p, ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], use_cuda=False)
    assert m.NeighConsensus.channels == [16, 1] and m.NeighConsensus.kernel_sizes == [3, 3]
    for k, v in src.state_dict().items():
        if "num_batches_tracked" in k:
            continue
        assert torch.equal(m.state_dict()[k], v), k


def test_checkpoint_roundtrip_and_best_copy(tmp_path):
    from ncnet_amd.engine.checkpoint import load_checkpoint, save_checkpoint
    f = str(tmp_path / "models" / "2024-01-01_00:00_checkpoint_adam.pth.tar")
    st = {"epoch": 1, "args": argparse.Namespace(a=1), "state_dict": OrderedDict(w=torch.ones(2)),
          "best_test_loss": 1.0, "optimizer": {}, "train_loss": np.ones(2), "test_loss": np.ones(2)}
    save_checkpoint(st, True, f)
    assert os.path.exists(f) and os.path.exists(str(tmp_path / "models" / "best_2024-01-01_00:00_checkpoint_adam.pth.tar"))
    ld = load_checkpoint(f)
    assert ld["args"].a == 1 and torch.equal(ld["state_dict"]["w"], torch.ones(2))
    assert np.array_equal(ld["test_loss"], np.ones(2))


def test_str_to_bool():
    from ncnet_amd.engine.checkpoint import str_to_bool
    assert str_to_bool("True") and str_to_bool("1") and not str_to_bool("no")
    with pytest.raises(argparse.ArgumentTypeError):
        str_to_bool("maybe")


def test_weak_loss_cpu_equals_reference_algorithm():
    """Feature reuse for the negative pass == the reference's second forward."""
    from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_weak_loss
    from ncnet_amd.engine.trainer import weak_loss
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    batch = {"source_image": torch.randn(3, 3, 96, 96), "target_image": torch.randn(3, 3, 96, 96)}
    l1 = weak_loss(m, batch)
    l1.backward()
    g1 = [p.grad.clone() for p in m.NeighConsensus.parameters()]
    m.zero_grad()
    l2 = reference_weak_loss(ReferenceAlgorithm(m), batch)
    l2.backward()
    g2 = [p.grad.clone() for p in m.NeighConsensus.parameters()]
    assert abs(float(l1) - float(l2)) < 1e-5
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-7)


def test_fold_frozen_bn_equivalence():
    from ncnet_amd.models.backbones import fold_frozen_bn, resnet_trunk
    torch.manual_seed(0)
    t = resnet_trunk("resnet101", "layer2").eval()
    for m in t.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
    f = fold_frozen_bn(t)
    x = torch.randn(1, 3, 64, 64)
    with torch.no_grad():
        assert torch.allclose(t(x), f(x), rtol=1e-4, atol=1e-4)


def test_frozen_resnet_plan_equivalence():
    """Pre-cast execution plan of the folded trunk == eager trunk (fp32, CPU)."""
    from ncnet_amd.models.backbones import FrozenResNetPlan, fold_frozen_bn, resnet_trunk
    torch.manual_seed(0)
    t = resnet_trunk("resnet101", "layer3").eval()
    for m in t.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
    plan = FrozenResNetPlan(fold_frozen_bn(t), torch.float32)
    x = torch.randn(1, 3, 80, 64)
    with torch.no_grad():
        r, p = t(x), plan(x)
    assert p.shape == r.shape
    assert ((p - r).norm() / r.norm()).item() < 1e-5


def test_fp8_correlation_cpu_path():
    from ncnet_amd.ops.correlation import FP8, FP8_FEAT_SCALE, correlation, l2norm_pack_fp8
    torch.manual_seed(0)
    f = torch.randn(2, 64, 5, 4)
    y = l2norm_pack_fp8(f)
    assert y.dtype == FP8 and y.shape == (2, 20, 64)
    c = correlation(y, y)
    cb = correlation(ref.feature_l2norm(f).reshape(2, 64, 20).transpose(1, 2),
                     ref.feature_l2norm(f).reshape(2, 64, 20).transpose(1, 2))
    assert float((c - cb).abs().max()) < 0.08
    assert abs(FP8_FEAT_SCALE - 16.0) < 1e-9


def test_extension_imports_when_built():
    """A built _C.so must import on CPU too (catches unresolved launcher symbols
    before a GPU run)."""
    from ncnet_amd.ops import _ext
    so = os.path.join(os.path.dirname(_ext.__file__), "..", "_C.so")
    if not os.path.exists(so):
        pytest.skip("extension not built")
    assert _ext.load() is not None


def test_trunk_prefetcher_cpu_fallback():
    """On CPU (and whenever the backbone is trainable) the prefetcher is off:
    take() runs the backbone in place and the loss equals weak_loss."""
    from ncnet_amd.engine.trainer import TrunkPrefetcher, weak_loss, weak_loss_from_features
    from ncnet_amd.models import ImMatchNet

    torch.manual_seed(0)
    model = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    model.eval()
    batch = {"source_image": torch.randn(2, 3, 64, 64), "target_image": torch.randn(2, 3, 64, 64)}
    pre = TrunkPrefetcher(model)
    assert not pre.enabled
    pre.submit(batch)
    with torch.no_grad():
        l1 = weak_loss_from_features(model, pre.take(batch))
        l2 = weak_loss(model, batch)
    assert torch.allclose(l1, l2, rtol=1e-6, atol=1e-9)
