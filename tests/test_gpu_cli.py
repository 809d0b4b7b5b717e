"""The command lines end to end on the MI355X (the CPU suite runs the same
flows on the torch oracles): train.py on synthetic pairs with checkpoint and
resume, eval_pf_pascal.py, eval_inloc.py (bf16 and fp8, the query-once /
batched-pano schedule) with the .mat contract, and the keypoint-transfer demo.
Every NC-Net op must dispatch to a HIP kernel: no torch fallback."""
import glob
import os

import numpy as np
import pytest

from ncnet_amd.ops import _ext

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("gpucli")
    old = os.getcwd()
    os.chdir(d)
    yield d
    os.chdir(old)


def test_train_resume_eval_gpu(workdir):
    import eval_pf_pascal
    import train
    before = _ext.DISPATCH["torch_fallback"]
    train.main(["--synthetic", "8", "--batch_size", "4", "--image_size", "128", "--num_epochs", "1",
                "--result-model-dir", "models"])
    cks = sorted(glob.glob("models/2*_checkpoint_adam.pth.tar"))
    assert cks
    train.main(["--synthetic", "8", "--batch_size", "4", "--image_size", "128", "--num_epochs", "2",
                "--resume", cks[0]])
    from ncnet_amd.engine.checkpoint import load_checkpoint
    assert load_checkpoint(cks[0])["epoch"] == 2
    stats = eval_pf_pascal.main(["--synthetic", "4", "--image_size", "128", "--checkpoint", cks[0]])
    assert stats["point_tnf"]["pck"].shape[0] == 4
    assert _ext.DISPATCH["torch_fallback"] == before
    assert _ext.DISPATCH["nc_bf16"] > 0


@pytest.mark.parametrize("fp8", [False, True])
def test_inloc_export_gpu(workdir, fp8):
    import eval_inloc
    from scipy.io import loadmat
    before = _ext.DISPATCH["nc_fused_k3"]
    args = ["--synthetic_queries", "1", "--n_panos", "3", "--image_size", "640", "--k_size", "2",
            "--output_dir", "m8" if fp8 else "m16"]
    out = eval_inloc.main(args + (["--fp8"] if fp8 else []))
    assert _ext.DISPATCH["nc_fused_k3"] > before                # (replays of the pair graph are not counted)
    m = loadmat(os.path.join(out, "1.mat"))["matches"]
    assert m.shape[:2] == (1, 3) and m.dtype == np.float64
    used = m[0, 0, :, 4] > 0
    assert used.sum() > 0
    xy = m[0, 0, used, :4]
    assert (xy > 0).all() and (xy < 1).all()


def test_point_transfer_demo_gpu(workdir):
    import point_transfer_demo
    out = os.path.join(workdir, "demo_gpu.png")
    acc = point_transfer_demo.main(["--synthetic", "--image_size", "240", "--out", out])
    assert os.path.exists(out) and 0.0 <= acc <= 1.0


def _train_one_step_like_bench():
    """The state bench.py leaves before its InLoc secondaries: cudnn.benchmark
    on, a headline-config training step through the Trainer (side streams,
    trunk prefetch, flat Adam)."""
    import torch
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import DistContext
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(dev).train()
    params = [p for p in m.parameters() if p.requires_grad]
    tr = Trainer(m, make_adam(params, 5e-4), DistContext(device=dev))
    pool = [{"source_image": torch.randn(2, 3, 400, 400, device=dev),
             "target_image": torch.randn(2, 3, 400, 400, device=dev)} for _ in range(2)]
    for i in range(2):
        tr.train_step(pool[i % 2], pool[(i + 1) % 2])
    torch.cuda.synchronize()


@pytest.mark.parametrize("nc_fp8", [False, True])
def test_pair_matcher_graph_equals_eager(nc_fp8, monkeypatch):
    """eval/inloc.py PairMatcher: the HIP-graph replay of correlation .. match
    extraction returns exactly the eager matches, for a fixed query and
    changing panos (static inputs re-filled per replay) -- captured in the
    bench process state (after training steps, cudnn.benchmark=True), and for
    the all-fp8 pipeline (fp8 correlation + fp8 Conv4d NC) too."""
    import torch
    from ncnet_amd.eval.inloc import PairMatcher, pair_matches
    from ncnet_amd.models import ImMatchNet
    old = torch.backends.cudnn.benchmark
    try:
        _train_one_step_like_bench()
        if nc_fp8:
            from tests.conftest import set_runtime
            set_runtime(monkeypatch, nc_fp8=True)
        torch.manual_seed(3)
        m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], relocalization_k_size=2,
                       half_precision=True, corr_dtype="fp8" if nc_fp8 else "bf16").cuda().eval()
        src = torch.randn(1, 3, 320, 416, device="cuda")
        panos = [torch.randn(1, 3, 320, 416, device="cuda") for _ in range(3)]
        pm = PairMatcher(m, 2)
        with torch.inference_mode():
            fq = m.extract(src)
            for t in panos:
                fp = m.extract(t)
                res, cnt = pm(fq[0], fq[1], fp[0], fp[1])
                got = res[:int(cnt)].clone()
                corr, delta = m.match_features(fq[0], fq[1], fp[0], fp[1])
                want = pair_matches(corr, delta, 2)
                assert torch.equal(got, want)
        assert pm.capture_error is None, pm.capture_error
        assert pm.graphed, "the pair graph was not captured"
    finally:
        torch.backends.cudnn.benchmark = old
