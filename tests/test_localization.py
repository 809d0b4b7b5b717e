"""InLoc localization back end (Python port of the reference's MATLAB side):
P3P / LO-RANSAC on synthetic cameras, pose errors, localization-rate curve,
tentative-correspondence construction."""
import numpy as np

from ncnet_amd.eval.localization import (DEFAULT_THRESHOLDS, angular_errors, evaluate_queries, localization_rate,
                                         p3p, p3p_ransac, pose_center, pose_distance, resize_longest,
                                         tentative_correspondences)


def _rand_pose(rng):
    A = rng.normal(size=(3, 3))
    Q, _ = np.linalg.qr(A)
    if np.linalg.det(Q) < 0:
        Q[:, 0] *= -1
    t = rng.normal(size=3)
    return np.hstack([Q, t[:, None]])


def _scene(rng, n, P):
    # points in front of the camera: sample in camera frame, map to world
    Xc = np.stack([rng.uniform(-2, 2, n), rng.uniform(-2, 2, n), rng.uniform(3, 8, n)])
    R, t = P[:, :3], P[:, 3:4]
    Xw = R.T @ (Xc - t)
    return Xc, Xw


def test_p3p_recovers_pose_exactly():
    rng = np.random.default_rng(1)
    for _ in range(20):
        P = _rand_pose(rng)
        Xc, Xw = _scene(rng, 3, P)
        sols = p3p(Xc, Xw)
        assert sols, "no P3P solution"
        err = min(np.abs(S - P).max() for S in sols)
        assert err < 1e-6


def test_p3p_ransac_with_outliers():
    rng = np.random.default_rng(2)
    P = _rand_pose(rng)
    Xc, Xw = _scene(rng, 200, P)
    rays = Xc / np.linalg.norm(Xc, axis=0)
    rays += rng.normal(scale=1e-4, size=rays.shape)
    out = rng.random(200) < 0.4                       # 40% outliers
    rays[:, out] = rng.normal(size=(3, out.sum()))
    rays[2, out] = np.abs(rays[2, out])
    Pe, inl = p3p_ransac(rays, Xw, np.radians(0.2), max_iters=2000)
    assert Pe is not None
    dpos, dori = pose_distance(P, Pe)
    assert dpos < 1e-2 and dori < 1e-2
    assert inl[~out].mean() > 0.95 and inl[out].mean() < 0.05
    assert np.all(angular_errors(Pe, rays[:, inl], Xw[:, inl]) < np.radians(0.2))


def test_pose_center_distance_and_rate_curve():
    P1 = np.hstack([np.eye(3), np.array([[1.0], [2.0], [3.0]])])
    assert np.allclose(pose_center(P1), [-1, -2, -3])
    th = np.radians(30)
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    P2 = np.hstack([Rz, np.array([[1.0], [2.0], [3.5]])])
    dpos, dori = pose_distance(P1, P2)
    assert abs(dori - th) < 1e-9
    assert dpos > 0
    rate = localization_rate([0.1, 0.5, 3.0, 0.2], np.radians([1, 2, 3, 20]))
    assert len(rate) == len(DEFAULT_THRESHOLDS) == 25
    # thresholds 0.25 -> only 0.1 qualifies (0.2 has 20 deg rotation error)
    k = int(np.flatnonzero(np.isclose(DEFAULT_THRESHOLDS, 0.25))[0])
    assert rate[k] == 0.25
    assert rate[-1] == 0.5
    pos, ori = evaluate_queries(
        [{"queryname": "a", "P": P1, "floor": "DUC1"}, {"queryname": "b", "P": P1, "floor": "DUC2"},
         {"queryname": "c", "P": P1, "floor": "DUC1"}],
        {"a": ("DUC1/x.jpg", P1), "b": ("DUC1/y.jpg", P1)})
    assert pos[0] == 0 and np.isinf(pos[1]) and np.isinf(pos[2])


def test_tentative_correspondences_geometry():
    rng = np.random.default_rng(3)
    hq, wq, hd, wd = 48, 64, 30, 40
    xyz = rng.normal(size=(hd, wd, 3))
    xyz[0, :, :] = np.nan                              # rows without depth are dropped
    m = np.zeros((6, 5))
    m[:, 0] = [0.1, 0.5, 0.9, 0.2, 0.3, 0.7]
    m[:, 1] = [0.2, 0.5, 0.8, 0.9, 0.1, 0.6]
    m[:, 2] = [0.5, 0.25, 0.75, 0.0, 0.6, 0.3]
    m[:, 3] = [0.5, 0.5, 0.9, 0.5, 0.0, 0.4]
    m[:, 4] = [0.9, 0.8, 0.1, 0.95, 0.99, 0.85]
    rays, X, xq, xd = tentative_correspondences(m, 0.75, (hq, wq), xyz, focal=100.0)
    keep = m[:, 4] > 0.75
    # match 4 hits DB row floor(0*30)=0 -> fixed to 1 -> NaN row -> dropped
    assert rays.shape[1] == keep.sum() - 1
    assert np.allclose(rays[2], 1.0)
    r0 = 0  # first kept match
    assert np.isclose(rays[0, r0], (wq * m[0, 0] - wq / 2) / 100.0)
    assert np.allclose(X[:, r0], xyz[int(np.floor(hd * 0.5)) - 1, int(np.floor(wd * 0.5)) - 1])


def test_resize_longest():
    img = np.zeros((100, 3000, 3), dtype=np.uint8)
    out = resize_longest(img, 1920)
    assert out.shape[1] == 1920 and out.shape[0] == 64
    assert resize_longest(img[:, :500]).shape == (100, 500, 3)
