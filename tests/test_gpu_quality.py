"""GPU: numerics of the inference precisions and training quality vs the fp32
reference algorithm (VERDICT r1 "prove training quality").  Longer runs of the
same code: scripts/train_quality.py, scripts/precision_agreement.py
(results in profiles/r2_quality/)."""
import os
import sys

import pytest
import torch

from ncnet_amd.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scripts"))


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def test_fp32_mode_matches_reference_algorithm():
    """corr_dtype='fp32' (fp32 trunk, bf16x3 correlation + NC on the MFMA
    kernels) reproduces the reference's fp32 computation: volume error two
    orders below the bf16 path's, identical best matches."""
    from ncnet_amd.data.datasets import synthetic_correspondence_batch
    from ncnet_amd.engine.reference_impl import ReferenceAlgorithm
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(DEV).eval()
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.1)
    alg = ReferenceAlgorithm(m, torch.float32)
    b = synthetic_correspondence_batch(2, 320, DEV, seed=3)
    with torch.inference_mode():
        r = alg(b)
        c16 = m(b)
        m.corr_dtype, m.compute_dtype = "fp32", torch.float32
        n0 = _ext.DISPATCH["nc_x3"]
        c32 = m(b)
        assert _ext.DISPATCH["nc_x3"] == n0 + 1
    e16, e32 = rl2(c16, r), rl2(c32, r)
    assert e32 < 2e-3 and e32 < e16 / 10, (e16, e32)
    V = r.shape[0]
    r3, c3 = r.reshape(V, 400, 400), c32.reshape(V, 400, 400)
    assert (r3.argmax(1) == c3.argmax(1)).float().mean() > 0.995


def test_training_tracks_fp32_reference():
    """40 steps of the HIP trainer (fp32-accurate NC: nc_precision='fp32') and of
    the fp32 reference algorithm from the same init on known-correspondence
    pairs with the random-init trunk, where the weak loss's signal is below bf16
    resolution (the bf16 default's loss stays at 0 and its PCK at ~0 here,
    profiles/r2_quality).  The dynamics are chaotic in this regime -- one
    reference run ends anywhere in PCK 0.04-0.64 depending on the last bits of
    its arithmetic -- so one HIP run cannot be compared with one reference
    run.  Over four seeds: the HIP loss decreases in every run, the model
    learns (mean PCK well above init) and its mean PCK is within 0.3 of the
    reference's mean (3-seed means were seen 0.2 apart in either direction;
    the bf16 default stays near 0 here)."""
    import train_quality
    runs = []
    for seed in (0, 1, 2, 3):
        res = train_quality.main(["--steps", "40", "--batch", "4", "--image-size", "240", "--eval-batches", "4",
                                  "--nc-precision", "fp32", "--seed", str(seed)])
        runs.append(res)
        s = res["summary"]
        assert s["loss_first_hip"] - s["loss_last_hip"] > 0, s
    mean = lambda k: sum(r[k] for r in runs) / len(runs)  # noqa: E731
    summary = {k: mean(k) for k in ("pck_init_hip", "pck_final_hip", "pck_final_ref")}
    print("training-quality over 4 seeds:", summary)
    assert summary["pck_final_hip"] > summary["pck_init_hip"] + 0.1, summary
    assert summary["pck_final_hip"] > summary["pck_final_ref"] - 0.3, summary


def _nc_std(m):
    from ncnet_amd.ops import reference as ref
    layers = m.NeighConsensus.conv_layers()
    return [ref.conv4d_weight_to_std(l.weight_ref()).detach() for l in layers], [l.bias.detach() for l in layers]


@pytest.fixture
def deterministic_trunk(monkeypatch):
    """Pin the operating point: native trunk kernels only (no per-shape
    timing-based hipBLASLt choice) and no MIOpen benchmark-mode solver search
    for the stem, whatever earlier tests in the session switched on."""
    from tests.conftest import set_runtime
    set_runtime(monkeypatch, trunk_conv="native")
    old = torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    yield
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = old


@pytest.mark.parametrize("fe_finetune", [0, 1])
def test_training_grads_vs_quantized_oracle(fe_finetune, deterministic_trunk):
    """End-to-end gradients of the fused training path (features reused for the
    rolled negatives, HIP correlation / MutualMatching / ij-encoded NC with the
    side-stream weight gradients) against its own math in float64 with bf16
    rounding at exactly the stored-bf16 points (engine/quantized_oracle.py), at
    a non-degenerate operating point (known-correspondence pairs, after three
    Adam steps).  fe_finetune=1 unfreezes the last layer3 bottleneck
    (train.py:60-63): the L2-norm, correlation and first-MutualMatching
    backward and the NC input gradient are then checked too, as the gradient
    w.r.t. the raw trunk features."""
    from ncnet_amd.data.datasets import synthetic_correspondence_batch
    from ncnet_amd.engine import quantized_oracle as qo
    from ncnet_amd.engine.trainer import make_adam, weak_loss
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.ops.correlation import l2norm_pack
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1]).to(DEV)
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.05)
    m.train()
    opt = make_adam([p for p in m.parameters() if p.requires_grad], 5e-4)
    # the operating point: three NC Adam steps with the trunk frozen.  (Training
    # the trunk here too makes the point itself run-dependent -- MIOpen's
    # backward-weight convolutions are not bitwise deterministic -- and with it
    # how many MutualMatching argmax near-ties the bf16 path and the oracle
    # resolve differently: measured 2.6e-3 .. 2.7e-2 NC gradient error over
    # runs of one build, profiles/r2_sanitizers/README.md.)
    for s in range(3):
        b = synthetic_correspondence_batch(2, 240, DEV, seed=s)
        opt.zero_grad(set_to_none=True)
        weak_loss(m, {"source_image": b["source_image"], "target_image": b["target_image"]}).backward()
        opt.step()
    if fe_finetune:
        for p in m.FeatureExtraction.model[-1][-1].parameters():
            p.requires_grad = True
    b = synthetic_correspondence_batch(2, 240, DEV, seed=7)
    imgs = torch.cat((b["source_image"], b["target_image"]))
    opt.zero_grad(set_to_none=True)
    if fe_finetune:
        raw = m.FeatureExtraction.trunk_forward(imgs, torch.bfloat16).detach().requires_grad_(True)
        f, hw = l2norm_pack(raw), tuple(raw.shape[-2:])
    else:
        with torch.no_grad():
            f, hw = m.extract(imgs)
    vols = m.weak_loss_volumes_from_features(f, hw, 2)
    G = torch.randn_like(vols)
    (vols * G).sum().backward()
    g_hip = [p.grad.detach().double().clone() for p in m.NeighConsensus.parameters()]
    ws, bs = _nc_std(m)
    ws = [w.double().requires_grad_(True) for w in ws]
    bs = [x.double().requires_grad_(True) for x in bs]
    if fe_finetune:
        raw64 = raw.detach().double().requires_grad_(True)
        ovols = qo.weak_loss_volumes(raw64, hw, 2, ws, bs, normalize=True)
    else:
        ovols = qo.weak_loss_volumes(f.detach(), hw, 2, ws, bs, normalize=False)
    (ovols * G.double()).sum().backward()
    errs = {"vols": rl2(vols, ovols)}
    o_grads = []
    for w, x in zip(ws, bs):
        o_grads += [w.grad, x.grad]
    # NC parameters are (weight, bias) per layer in module order; the oracle's are std-layout weights
    from ncnet_amd.ops import reference as ref
    for i, (gh, go) in enumerate(zip(g_hip, o_grads)):
        if gh.dim() == 6:
            go = ref.conv4d_weight_from_std(go)
        errs[f"nc{i}"] = rl2(gh, go)
    if fe_finetune:
        errs["d_raw_features"] = rl2(raw.grad, raw64.grad)
    print("quantized-oracle errors:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["vols"] < 2e-3, errs
    # continuous data: the NC gradient error is set by ReLU-mask flips and
    # MutualMatching argmax near-ties (an L2 error ~ sqrt(flip rate)), measured
    # 2.6e-3 .. 2.7e-2 over runs of one build (above).  The kernel-level check
    # at 1e-3 runs on exactly representable data, where nothing flips:
    # tests/test_gpu_kernels.py::test_fast1x_stack_vs_quantized_oracle.
    assert max(v for k, v in errs.items() if k.startswith("nc")) < 3e-2, errs
    # the raw-feature gradient crosses the first MutualMatching's argmax: an
    # argmax near-tie resolved differently by the bf16 path and the oracle
    # moves it discretely, and which ties exist depends on the operating point
    # (the three Adam steps above; a different fp32 summation order of the
    # weight gradients alone moved it 2.2e-2 -> 2.8e-2)
    assert errs.get("d_raw_features", 0.0) < 6e-2, errs
