"""Dense pose verification pieces (ncnet_amd/eval/pose_verification.py):
z-buffer rendering, in-painting, dense SIFT, scoring and re-ranking, InLoc
scan naming / transformation parsing.  CPU only."""
import math

import numpy as np
import pytest
import torch

from ncnet_amd.eval import pose_verification as pv


def test_zbuffer_keeps_nearest_point():
    xyz = torch.tensor([[0.0, 0.0, 2.0], [0.0, 0.0, 5.0], [0.3, 0.0, 1.0], [0.0, 0.0, -1.0]], dtype=torch.float64)
    rgb = torch.tensor([[10.0] * 3, [20.0] * 3, [30.0] * 3, [40.0] * 3])
    K = torch.tensor([[10.0, 0, 5], [0, 10.0, 5], [0, 0, 1]], dtype=torch.float64)
    KP = K @ torch.cat([torch.eye(3, dtype=torch.float64), torch.zeros(3, 1, dtype=torch.float64)], 1)
    img, xyz_img = pv.points_to_perspective(rgb, xyz, KP, 10, 10)
    assert float(img[5, 5, 0]) == 10.0            # the z=2 point hides the z=5 one; z<0 dropped
    assert float(img[5, 8, 0]) == 30.0            # u = floor(10 * 0.3 / 1 + 5) = 8
    assert int((~torch.isnan(img[..., 0])).sum()) == 2
    assert torch.allclose(xyz_img[5, 5], torch.tensor([0.0, 0.0, 2.0]))


def test_inpaint_fills_and_keeps_known():
    img = torch.arange(25.0).view(5, 5)
    holes = img.clone()
    holes[1:4, 1:4] = float("nan")
    out = pv.inpaint_nans(holes)
    assert torch.isfinite(out).all()
    assert torch.equal(out[0], img[0]) and torch.equal(out[:, 0], img[:, 0])
    assert abs(float(out[2, 2]) - 12.0) < 1.0      # a linear ramp is harmonic: reconstructed closely


def test_dense_sift_shapes_and_normalisation():
    g = torch.Generator().manual_seed(0)
    img = torch.rand(64, 80, generator=g)
    f, d = pv.dense_sift(img)
    assert d.shape[0] == 128 and f.shape == (2, d.shape[1]) and d.shape[1] > 0
    n = d.norm(dim=0)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-4)
    assert float(d.max()) < 0.25                  # clamped at 0.2 before the final renormalisation
    # frame step 4 px, first centre at 2*size - 1
    assert float(f[0, 1] - f[0, 0]) == 4.0 and float(f[0, 0]) == 15.0
    # a constant image has no gradients: all-zero descriptors
    f0, d0 = pv.dense_sift(torch.full((64, 80), 0.5))
    assert float(d0.abs().max()) == 0.0
    # RootSIFT columns have unit L2 norm after sqrt of L1-normalised values
    r = pv.root_sift(d)
    assert torch.allclose(r.norm(dim=0), torch.ones(r.shape[1]), atol=1e-4)


def _scene(seed=0):
    rng = np.random.default_rng(seed)
    K = np.array([[300.0, 0, 160], [0, 300.0, 120], [0, 0, 1]])
    vv, uu = np.meshgrid(np.arange(0, 240, 1.0), np.arange(0, 320, 1.0), indexing="ij")
    z = 4.0 + 0.5 * np.sin(uu / 40.0)
    X = (np.linalg.solve(K, np.stack([uu.ravel(), vv.ravel(), np.ones(uu.size)])) * z.ravel()).T
    tex = (np.sin(3 * X[:, 0]) + np.cos(4 * X[:, 1]) + 2) / 4 * 255
    rgb = np.repeat(tex[:, None], 3, 1)
    P = np.hstack([np.eye(3), np.zeros((3, 1))])
    img, _ = pv.points_to_perspective(torch.tensor(rgb), torch.tensor(X), torch.tensor(K @ P), 240, 320)
    q = pv.inpaint_nans(pv.rgb2gray(img)).numpy()
    return np.repeat(q[..., None], 3, 2), rgb, X, P, 300.0, rng


def test_pv_score_prefers_true_pose_and_rerank():
    qimg, rgb, X, P, f, _ = _scene()
    a = math.radians(8.0)
    R = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    P_bad = np.hstack([R, np.array([[0.4], [0.0], [0.0]])])
    s_true, synth, flag, errmap = pv.pv_score(qimg, rgb, X, P, f, ds=0.25)
    s_bad = pv.pv_score(qimg, rgb, X, P_bad, f, ds=0.25)[0]
    assert s_true > 2 * s_bad > 0
    assert synth.shape == (60, 80, 3) and flag.dtype == bool and errmap.ndim == 2
    assert pv.pv_score(qimg, rgb, X, np.full((3, 4), np.nan), f)[0] == 0.0
    ranked, sc = pv.rerank([("bad", P_bad), ("good", P)], [s_bad, s_true])
    assert ranked[0][0] == "good" and sc == sorted(sc, reverse=True)


def test_inloc_scan_names_and_transformation(tmp_path):
    floor, scene, scan = pv.parse_cutout_name("DUC1/024/DUC_cutout_024_30_0.jpg")
    assert (floor, scene, scan) == ("DUC1", "DUC", "024")
    sp, tp = pv.scan_paths("DUC2/117/DUC_cutout_117_0_-30.jpg", "/scans")
    assert sp == "/scans/DUC2/DUC_scan_117.ptx.mat"
    assert tp == "/scans/DUC2/transformations/DUC_trans_117.txt"
    with pytest.raises(ValueError):
        pv.parse_cutout_name("not/a/cutout.jpg")
    T = np.arange(16, dtype=float).reshape(4, 4)
    p = tmp_path / "t.txt"
    p.write_text("header line\nscan to global:\n" + "\n".join(" ".join(str(v) for v in r) for r in T) + "\n")
    assert np.array_equal(pv.load_transformation(str(p)), T)
