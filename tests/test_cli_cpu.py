"""End-to-end CLI runs on CPU at tiny sizes (train -> checkpoint -> resume ->
PF-Pascal eval -> InLoc export with the .mat contract)."""
import glob
import os

import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    old = os.getcwd()
    os.chdir(d)
    yield d
    os.chdir(old)


def test_train_resume_eval(workdir):
    import eval_pf_pascal
    import train
    train.main(["--synthetic", "4", "--batch_size", "2", "--image_size", "64", "--ncons_kernel_sizes", "3", "3",
                "--ncons_channels", "16", "1", "--num_epochs", "1", "--result-model-dir", "models"])
    cks = sorted(glob.glob("models/2*_checkpoint_adam.pth.tar"))
    assert cks and os.path.exists(os.path.join("models", "best_" + os.path.basename(cks[0])))
    from ncnet_amd.engine.checkpoint import load_checkpoint
    ck = load_checkpoint(cks[0])
    assert ck["epoch"] == 1 and ck["args"].ncons_channels == [16, 1]
    assert set(ck) >= {"epoch", "args", "state_dict", "best_test_loss", "optimizer", "train_loss", "test_loss"}
    train.main(["--synthetic", "4", "--batch_size", "2", "--image_size", "64", "--num_epochs", "2", "--resume", cks[0]])
    ck2 = load_checkpoint(cks[0])
    assert ck2["epoch"] == 2
    stats = eval_pf_pascal.main(["--synthetic", "2", "--image_size", "64", "--checkpoint", cks[0]])
    assert stats["point_tnf"]["pck"].shape == (2, 1)


def test_inloc_export_contract(workdir):
    import eval_inloc
    from scipy.io import loadmat
    out = eval_inloc.main(["--synthetic_queries", "1", "--n_panos", "2", "--image_size", "256", "--k_size", "2",
                           "--output_dir", "m"])
    assert os.path.basename(out) == "synthetic_shortlist_SZ_NEW_256_K_2_BOTHDIRS_SOFTMAX"
    d = loadmat(os.path.join(out, "1.mat"))
    m = d["matches"]
    n = 2 * int(256 * 0.0625 / 2 * np.floor(256 * 0.0625 / 2 * 0.75))
    assert m.shape == (1, 2, n, 5) and m.dtype == np.float64
    used = m[0, 0, :, 4] > 0
    xy = m[0, 0, used, :4]
    assert (xy > 0).all() and (xy < 1).all()
    # de-duplicated and in lexicographic (xA, yA, xB, yB) order like np.unique
    rows = [tuple(r) for r in xy]
    assert rows == sorted(set(rows))


def test_inloc_export_square_grows_n(workdir):
    """A square query pools to an 8 x 8 grid at 256 px: more unique matches than
    the reference's 4:3 N (2 * 8 * 6 = 96).  The export grows the array instead
    of silently dropping rows (the reference raises on the overflow)."""
    import eval_inloc
    from scipy.io import loadmat
    out = eval_inloc.main(["--synthetic_queries", "1", "--n_panos", "1", "--image_size", "256", "--k_size", "2",
                           "--synthetic_hw", "512", "512", "--output_dir", "msq"])
    m = loadmat(os.path.join(out, "1.mat"))["matches"]
    used = m[0, 0, :, 4] > 0
    n_ref = 2 * 8 * 6
    assert used.sum() > n_ref and m.shape[2] == used.sum()
    rows = [tuple(r) for r in m[0, 0, used, :4]]
    assert rows == sorted(set(rows))


def test_point_transfer_demo(workdir):
    import point_transfer_demo
    out = os.path.join(workdir, "demo.png")
    acc = point_transfer_demo.main(["--synthetic", "--image_size", "160", "--out", out])
    assert os.path.exists(out) and 0.0 <= acc <= 1.0


def test_inloc_localize_synthetic(workdir):
    """P3P LO-RANSAC on the shortlist's top-1 pano (whose matches support a
    wrong pose in the synthetic scene) fails; dense pose verification
    re-ranks the candidates and recovers every query."""
    import inloc_localize
    args = ["--synthetic", "2", "--ransac_iters", "2000", "--out", os.path.join(workdir, "poses.npz")]
    est, rate = inloc_localize.main(args)
    assert len(est) == 2 and rate[-1] == 0.0
    assert os.path.exists(os.path.join(workdir, "poses.npz"))
    est_pv, rate_pv = inloc_localize.main(args + ["--pv", "--plot", os.path.join(workdir, "curves.png")])
    assert len(est_pv) == 2 and rate_pv[-1] == 1.0
    assert os.path.exists(os.path.join(workdir, "curves.png"))
    assert os.path.exists("error_NCNet_PV.txt")


def test_inloc_localize_parallel_cached(workdir):
    """Pair tasks on 2 spawned workers match the serial run exactly; a rerun
    with the per-pair cache recomputes nothing and returns the same poses."""
    import numpy as np
    import inloc_localize
    cache = os.path.join(workdir, "cache")
    base = ["--synthetic", "2", "--ransac_iters", "500", "--pv", "--out", os.path.join(workdir, "p.npz")]
    est1, _ = inloc_localize.main(base + ["--workers", "1"])
    est2, _ = inloc_localize.main(base + ["--workers", "2", "--cache_dir", cache])
    n_pnp = sum(len(f) for _, _, f in os.walk(os.path.join(cache, "pnp")))
    n_pv = sum(len(f) for _, _, f in os.walk(os.path.join(cache, "pv")))
    assert n_pnp == 2 * 3 and n_pv == 2 * 3
    stamp = {os.path.join(d, f): os.path.getmtime(os.path.join(d, f)) for d, _, fs in os.walk(cache) for f in fs}
    est3, _ = inloc_localize.main(base + ["--workers", "2", "--cache_dir", cache])
    assert stamp == {os.path.join(d, f): os.path.getmtime(os.path.join(d, f)) for d, _, fs in os.walk(cache) for f in fs}
    # a rerun with another threshold must not reuse the cached poses / scores
    inloc_localize.main(base + ["--workers", "1", "--cache_dir", cache, "--thr", "0.5"])
    # (PV scores are keyed by the pose they scored: reused only for an identical P)
    pnp = [k for k in stamp if os.sep + "pnp" + os.sep in k]
    assert len(pnp) == 6 and all(os.path.getmtime(k) != stamp[k] for k in pnp)
    for e in (est2, est3):
        assert est1.keys() == e.keys()
        for k in est1:
            assert est1[k][0] == e[k][0]
            np.testing.assert_array_equal(est1[k][1], e[k][1])


def test_reference_refposes_parse():
    """The reference's own GT pose file (MATLAB v5, read with scipy.io.loadmat)."""
    import inloc_localize
    path = "/root/reference/lib_matlab/DUC_refposes_all.mat"
    if not os.path.exists(path):
        pytest.skip("reference GT poses not present")
    refs = inloc_localize.load_refposes(path)
    assert len(refs) == 198 + 131
    assert refs[0]["P"].shape == (3, 4) and refs[0]["floor"] == "DUC1"


def test_inloc_export_volume_parallel_torchrun(workdir):
    """eval_inloc.py --volume_parallel under torchrun (2 ranks, gloo): every
    pair's volume sharded over both ranks; the exported matches equal the
    single-process export."""
    import subprocess
    import sys

    import eval_inloc
    from scipy.io import loadmat
    common = ["--synthetic_queries", "1", "--n_panos", "2", "--image_size", "256", "--k_size", "2"]
    single = eval_inloc.main(common + ["--output_dir", "single"])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29733", os.path.join(root, "eval_inloc.py")] + common + [
           "--output_dir", "vp", "--volume_parallel"]
    out = subprocess.run(cmd, cwd=str(workdir), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    a = loadmat(os.path.join(single, "1.mat"))["matches"]
    b = loadmat(os.path.join("vp", os.path.basename(single), "1.mat"))["matches"]
    assert a.shape == b.shape
    assert np.allclose(a, b, rtol=1e-5, atol=1e-7)
