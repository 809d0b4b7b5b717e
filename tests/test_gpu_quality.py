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


# bounds just above the errors measured at these four operating points by
# scripts/oracle_tolerance.py (profiles/r5/quality/; one build reproduces them
# bitwise; the per-layer metric joins each layer's weight and bias gradients):
#   frozen trunk:  layer error <= 8.2e-3 (per-tensor NC error <= 1.4e-2 in an
#                  earlier build whose different wgrad summation order moved
#                  the operating points), volumes <= 3.4e-4;
#   fe_finetune:   layer error 4.6e-3 .. 1.9e-2, volumes <= 4.9e-4, raw-feature
#                  gradient <= 4.6e-2; a first-MutualMatching near-tie point
#                  reached 3.9e-2 .. 5.1e-2 per NC tensor in the earlier build;
#                  nc_any (the worst of the four points) sits just above what
#                  this build measures, so a regression at one point fails
ORACLE_POINTS = (0, 10, 20, 30)
ORACLE_TOL = {0: {"vols": 5e-4, "nc": 2e-2, "nc_any": 2e-2},
              1: {"vols": 1e-3, "nc": 2.5e-2, "nc_any": 3e-2, "d_raw": 6e-2}}


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
    rounding at exactly the stored-bf16 points (engine/quantized_oracle.py
    training_grad_errors), at four non-degenerate operating points (known-
    correspondence pairs, after three Adam steps with the trunk frozen).
    fe_finetune=1 unfreezes the last layer3 bottleneck (train.py:60-63): the
    L2-norm, correlation and first-MutualMatching backward and the NC input
    gradient are then checked too, as the gradient w.r.t. the raw trunk
    features.  One point is run twice: a build must reproduce itself bitwise
    (measured: it does, profiles/r5/quality/oracle_tolerance.json)."""
    from ncnet_amd.engine.quantized_oracle import training_grad_errors
    runs = {s: training_grad_errors(fe_finetune=fe_finetune, point_seed=s) for s in ORACLE_POINTS}
    again = training_grad_errors(fe_finetune=fe_finetune, point_seed=ORACLE_POINTS[0])
    for s, e in runs.items():
        print(f"point {s}: quantized-oracle errors:", {k: f"{v:.2e}" for k, v in e.items()})
    assert runs[ORACLE_POINTS[0]] == again, (runs[ORACLE_POINTS[0]], again)
    nc = sorted(max(v for k, v in e.items() if k.startswith("layer")) for e in runs.values())
    vols = max(e["vols"] for e in runs.values())
    tol = ORACLE_TOL[fe_finetune]
    assert vols < tol["vols"], runs
    # continuous data: the NC gradient error is set by ReLU-mask flips and
    # MutualMatching argmax near-ties (an L2 error ~ sqrt(flip rate)).  Frozen
    # trunk: every point within tol["nc"].  fe_finetune: the oracle recomputes
    # the correlation from the raw features in fp64, so a first-MutualMatching
    # near-tie can flip between the two -- typical points stay within
    # tol["nc"], one of the four measured ones reached 5.1e-2 (tol["nc_any"]).
    # The kernel-level check at 1e-3 runs on exactly representable data, where
    # nothing flips: tests/test_gpu_kernels.py::test_fast1x_stack_vs_quantized_oracle.
    assert nc[-2] < tol["nc"] and nc[-1] < tol["nc_any"], (nc, runs)
    if fe_finetune:
        # the raw-feature gradient crosses the first MutualMatching's argmax
        d_raw = max(e["d_raw_features"] for e in runs.values())
        assert d_raw < tol["d_raw"], runs
