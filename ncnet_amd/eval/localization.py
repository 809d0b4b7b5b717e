"""InLoc localization back end in Python (the MATLAB side of the reference).

The reference hands ``matches/<exp>/<q>.mat`` to MATLAB scripts built on the
external InLoc_demo toolbox.  This module provides the
pieces that live in the reference repository itself, so the whole
match -> pose -> localization-rate chain can run without MATLAB:

* ``tentative_correspondences``: score threshold + optional subsampling of one
  query/pano match list, query rays from the intrinsics, DB 3D points looked
  up in the cutout's XYZ map and moved to global coordinates, NaN points
  dropped (lib_matlab/parfor_NC4D_PE_pnponly.m:13-73).
* ``p3p`` + ``p3p_ransac``: calibrated absolute pose from 3 ray/point pairs
  (Grunert's quartic) inside LO-RANSAC with an angular inlier test -- the role
  of InLoc_demo's ``ht_lo_ransac_p3p`` (parfor_NC4D_PE_pnponly.m:77).
* ``pose_center`` / ``pose_distance``: camera centre and (position, rotation
  angle) error between two [R|t] poses (lib_matlab/p2c.m, p2dist.m).
* ``localization_rate``: fraction of queries localized within each distance
  threshold with rotation error <= 10 deg, thresholds [0:0.0625:1,
  1.125:0.125:2] m (lib_matlab/ht_plotcurve_WUSTL.m:70-82), and
  ``evaluate_queries`` for the per-floor top-1 check (:20-67).
* ``resize_longest``: longest side <= 1920 px (lib_matlab/at_imageresize_nc4d.m).

Dense pose verification (synthetic view rendering + dense SIFT, M4-M6) is in
``pose_verification.py``; match / curve plots (M7, M11) in ``utils/plot.py``.
"""
from __future__ import annotations

import numpy as np

DEFAULT_THRESHOLDS = np.concatenate([np.arange(0, 1 + 1e-9, 0.0625), np.arange(1.125, 2 + 1e-9, 0.125)])


# ---------------------------------------------------------------------------
def pose_center(P: np.ndarray) -> np.ndarray:
    """Camera centre C = -R^T t of P = [R | t] (p2c.m)."""
    P = np.asarray(P, dtype=np.float64)
    return -P[:3, :3].T @ P[:3, 3]


def pose_distance(P1: np.ndarray, P2: np.ndarray):
    """(position error, rotation angle in radians) between two [R|t] poses (p2dist.m)."""
    P1, P2 = np.asarray(P1, np.float64), np.asarray(P2, np.float64)
    dpos = float(np.linalg.norm(pose_center(P1) - pose_center(P2)))
    R = np.linalg.solve(P1[:3, :3], P2[:3, :3])
    c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    return dpos, float(np.arccos(c))


def localization_rate(pos_err, ori_err_rad, max_ori_deg: float = 10.0, thresholds=DEFAULT_THRESHOLDS):
    """Rate of queries with position error < threshold and rotation error <=
    max_ori_deg, for every threshold (ht_plotcurve_WUSTL.m:70-82)."""
    pos = np.asarray(pos_err, np.float64).copy()
    ori = np.degrees(np.asarray(ori_err_rad, np.float64))
    pos[ori > max_ori_deg] = np.inf
    thr = np.asarray(thresholds, np.float64)
    return (pos[:, None] < thr[None, :]).sum(0) / max(1, pos.size)


def evaluate_queries(ref_list, estimates):
    """Per-query top-1 errors with the floor check of ht_plotcurve_WUSTL.m:20-67.

    ref_list: iterable of dicts {queryname, P, floor}; estimates: dict
    queryname -> (top1 database name 'FLOOR/...', P or None).  Missing,
    wrong-floor or NaN poses count as infinite error."""
    pos, ori = [], []
    for r in ref_list:
        est = estimates.get(r["queryname"])
        if est is None:
            pos.append(np.inf), ori.append(np.inf)
            continue
        dbname, P = est
        floor_ok = str(dbname).split("/")[0] == r["floor"]
        if not floor_ok or P is None or np.isnan(np.asarray(P, np.float64)[0, 0]):
            pos.append(np.inf), ori.append(np.inf)
            continue
        dp, do = pose_distance(r["P"], P)
        pos.append(dp), ori.append(do)
    return np.asarray(pos), np.asarray(ori)


# ---------------------------------------------------------------------------
def tentative_correspondences(matches: np.ndarray, thr: float, q_size, xyz_cut: np.ndarray, focal: float,
                              P_after: np.ndarray | None = None, n_subsample: int | None = None, rng=None):
    """One query/pano match list -> (query rays [3,N], DB 3D points [3,N], query px [2,N], DB px [2,N]).

    matches: [N, 5] (xA, yA, xB, yB, score) in [0, 1] image coordinates
    (eval_inloc.py output); q_size = (H, W) of the query; xyz_cut [H, W, 3] the
    cutout's 3D map; P_after (3x4 or 4x4) the scan-to-global transform."""
    M = np.asarray(matches, np.float64).reshape(-1, 5)
    keep = M[:, 4] > thr
    f1, f2 = M[keep, 0:2].T.copy(), M[keep, 2:4].T.copy()
    if n_subsample is not None:
        rng = np.random.default_rng() if rng is None else rng
        sel = rng.permutation(f1.shape[1])[: min(f1.shape[1], n_subsample)]
        f1, f2 = f1[:, sel], f2[:, sel]
    hq, wq = q_size
    hd, wd = xyz_cut.shape[:2]
    xq = np.stack([wq * f1[0], hq * f1[1]])
    xd = np.stack([np.floor(wd * f2[0]), np.floor(hd * f2[1])])
    xd[xd == 0] = 1                                   # MATLAB 1-based "fix zeros"
    xd[0] = np.minimum(xd[0], wd)
    xd[1] = np.minimum(xd[1], hd)
    K = np.array([[focal, 0, wq / 2.0], [0, focal, hq / 2.0], [0, 0, 1.0]])
    rays = np.linalg.solve(K, np.vstack([xq, np.ones((1, xq.shape[1]))]))
    rr, cc = xd[1].astype(int) - 1, xd[0].astype(int) - 1
    X = xyz_cut[rr, cc].T.astype(np.float64)           # [3, N]
    if P_after is not None:
        Pa = np.asarray(P_after, np.float64)
        X = Pa[:3, :3] @ X + Pa[:3, 3:4]
    ok = ~np.isnan(X).any(0)
    return rays[:, ok], X[:, ok], xq[:, ok], xd[:, ok]


def _rigid_from_points(Xw: np.ndarray, Xc: np.ndarray):
    """R, t with Xc = R Xw + t (Kabsch / Horn, columns are points)."""
    mw, mc = Xw.mean(1, keepdims=True), Xc.mean(1, keepdims=True)
    H = (Xw - mw) @ (Xc - mc).T
    U, _, Vt = np.linalg.svd(H)
    D = np.diag([1.0, 1.0, np.sign(np.linalg.det(Vt.T @ U.T))])
    R = Vt.T @ D @ U.T
    return R, (mc - R @ mw).ravel()


def p3p(f: np.ndarray, X: np.ndarray):
    """Calibrated absolute pose from 3 bearing vectors f [3,3] (columns) and
    world points X [3,3]: Grunert's quartic (Haralick et al. 1994).  Returns a
    list of 3x4 [R|t] candidates (X_cam = R X + t)."""
    f = f / np.linalg.norm(f, axis=0, keepdims=True)
    X1, X2, X3 = X[:, 0], X[:, 1], X[:, 2]
    a2, b2, c2 = np.sum((X2 - X3) ** 2), np.sum((X1 - X3) ** 2), np.sum((X1 - X2) ** 2)
    if min(a2, b2, c2) < 1e-12:
        return []
    ca, cb, cg = f[:, 1] @ f[:, 2], f[:, 0] @ f[:, 2], f[:, 0] @ f[:, 1]
    p = (a2 - c2) / b2
    q = (a2 + c2) / b2
    A4 = (p - 1) ** 2 - 4 * c2 / b2 * ca ** 2
    A3 = 4 * (p * (1 - p) * cb - (1 - q) * ca * cg + 2 * c2 / b2 * ca ** 2 * cb)
    A2 = 2 * (p ** 2 - 1 + 2 * p ** 2 * cb ** 2 + 2 * (b2 - c2) / b2 * ca ** 2 - 4 * q * ca * cb * cg
              + 2 * (b2 - a2) / b2 * cg ** 2)
    A1 = 4 * (-p * (1 + p) * cb + 2 * a2 / b2 * cg ** 2 * cb - (1 - q) * ca * cg)
    A0 = (1 + p) ** 2 - 4 * a2 / b2 * cg ** 2
    out = []
    for v in np.roots([A4, A3, A2, A1, A0]):
        if abs(v.imag) > 1e-6 * max(1.0, abs(v.real)):
            continue
        v = v.real
        den = 2 * (cg - v * ca)
        if abs(den) < 1e-12:
            continue
        u = ((-1 + p) * v ** 2 - 2 * p * cb * v + 1 + p) / den
        s1sq = b2 / (1 + v ** 2 - 2 * v * cb)
        if s1sq <= 0 or u <= 0 or v <= 0:
            continue
        s1 = np.sqrt(s1sq)
        Xc = f * np.array([s1, u * s1, v * s1])
        R, t = _rigid_from_points(X, Xc)
        out.append(np.hstack([R, t[:, None]]))
    return out


def angular_errors(P: np.ndarray, rays: np.ndarray, X: np.ndarray) -> np.ndarray:
    """Angle between each observed ray and the direction of R X + t (inf behind the camera)."""
    Y = P[:3, :3] @ X + P[:3, 3:4]
    fn = rays / np.linalg.norm(rays, axis=0, keepdims=True)
    yn = Y / np.maximum(np.linalg.norm(Y, axis=0, keepdims=True), 1e-12)
    c = np.clip((fn * yn).sum(0), -1.0, 1.0)
    ang = np.arccos(c)
    ang[Y[2] <= 0] = np.inf
    return ang


def p3p_ransac(rays: np.ndarray, X: np.ndarray, thr_rad: float, max_iters: int = 10000, confidence: float = 0.999,
               lo_iters: int = 20, rng=None):
    """LO-RANSAC over P3P with an angular inlier threshold.  Returns (P 3x4 or
    None, inlier mask).  Local optimisation: minimal re-samples drawn from the
    current inliers (kept when they add inliers)."""
    rng = np.random.default_rng(0) if rng is None else rng
    n = rays.shape[1]
    best_P, best_in = None, np.zeros(n, dtype=bool)
    if n < 3:
        return None, best_in
    it, need = 0, max_iters
    while it < min(need, max_iters):
        it += 1
        idx = rng.choice(n, 3, replace=False)
        for P in p3p(rays[:, idx], X[:, idx]):
            inl = angular_errors(P, rays, X) < thr_rad
            if inl.sum() > best_in.sum():
                best_P, best_in = P, inl
                for _ in range(lo_iters):       # local optimisation on the inliers
                    ii = np.flatnonzero(best_in)
                    if ii.size < 4:
                        break
                    sub = rng.choice(ii, 3, replace=False)
                    for P2 in p3p(rays[:, sub], X[:, sub]):
                        inl2 = angular_errors(P2, rays, X) < thr_rad
                        if inl2.sum() > best_in.sum():
                            best_P, best_in = P2, inl2
                w = best_in.mean()
                if w > 0:
                    need = int(np.ceil(np.log(1 - confidence) / np.log(max(1e-12, 1 - w ** 3))))
    return best_P, best_in


# ---------------------------------------------------------------------------
def resize_longest(img: np.ndarray, imax: int = 1920) -> np.ndarray:
    """Downscale so that the longest side is <= imax (at_imageresize_nc4d.m)."""
    h, w = img.shape[:2]
    if max(h, w) <= imax:
        return img
    from PIL import Image

    if h > w:
        size = (max(1, round(w * imax / h)), imax)
    else:
        size = (imax, max(1, round(h * imax / w)))
    return np.asarray(Image.fromarray(img).resize(size, Image.BICUBIC))
