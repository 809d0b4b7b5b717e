#!/usr/bin/env python
"""InLoc pose estimation from NC-Net matches (the reference's MATLAB driver
compute_densePE_NCNet.m + ir_top100_NC4D_localization_pnponly.m +
parfor_NC4D_PE_pnponly.m, in Python on ncnet_amd.eval.localization).

For each query and each of its top-N shortlisted cutouts: threshold the
matches written by eval_inloc.py (score > --thr), build query rays and cutout
3D points, run P3P LO-RANSAC (--pnp_thr degrees), keep P and inliers.  The
query pose is the one of the top-1 cutout (reference behaviour) or, with
--rerank inliers, of the cutout with most inliers.  With --refposes (the
reference's lib_matlab/DUC_refposes_all.mat) it prints the localization rate
curve (ht_plotcurve_WUSTL.m) and writes error_<name>.txt.

--pv adds dense pose verification (ht_top10_NC4D_PV_localization.m,
at_pv_wrapper.m, parfor_nc4d_PV.m; ncnet_amd/eval/pose_verification.py): each
top-N pose is scored by rendering the cutout's scan (--scan_dir, InLoc
``<floor>/<scene>_scan_<id>.ptx.mat`` + ``transformations/``) at that pose and
comparing dense RootSIFT with the query image (--query_dir); the candidates are
re-ranked by that score ('InLoc + NCNet').  --plot writes the localization
curves of both methods (generate_ncnet_plot.m).

Inputs on disk (InLoc layout): --cutout_dir/<dbname>.mat with 'XYZcut'
[H,W,3]; optional --trans_dir/<dbname>.txt holding the 4x4 (or 3x4)
scan-to-global matrix.  --synthetic N builds a fake scene to smoke-test the
whole chain (including scans and query images for --pv).
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.eval.inloc import load_shortlist  # noqa: E402
from ncnet_amd.eval.localization import (DEFAULT_THRESHOLDS, evaluate_queries, localization_rate,  # noqa: E402
                                         p3p_ransac, tentative_correspondences)
from ncnet_amd.eval import pose_verification as pv  # noqa: E402


def _loadmat(path):
    from scipy.io import loadmat   # plain MATLAB v5 reader; executes nothing from the file
    return loadmat(path, squeeze_me=False)


def load_refposes(path: str):
    """DUC_refposes_all.mat (lib_matlab) -> [{queryname, P (3x4), floor}] (DUC1 then DUC2)."""
    m = _loadmat(path)
    refs = []
    for key, floor in (("DUC1_RefList", "DUC1"), ("DUC2_RefList", "DUC2")):
        for e in m[key].reshape(-1):
            refs.append({"queryname": str(np.asarray(e["queryname"]).reshape(-1)[0]),
                         "P": np.asarray(e["P"], np.float64), "floor": floor})
    return refs


def localize_query(q_matches: np.ndarray, db_names, q_size, args, rng):
    """q_matches [1, n_panos, N, 5] -> list of (dbname, P or None, n_inliers)."""
    out = []
    for jj, dbname in enumerate(db_names[: args.pnp_topN]):
        xyz_path = os.path.join(args.cutout_dir, dbname + ".mat")
        if not os.path.exists(xyz_path) or jj >= q_matches.shape[1]:
            out.append((dbname, None, 0))
            continue
        xyz = _loadmat(xyz_path)["XYZcut"].astype(np.float64)
        P_after = None
        if args.trans_dir:
            tp = os.path.join(args.trans_dir, dbname + ".txt")
            if os.path.exists(tp):
                P_after = np.loadtxt(tp)
        rays, X, _, _ = tentative_correspondences(q_matches[0, jj], args.thr, q_size, xyz, args.focal, P_after,
                                                  args.n_subsample, rng)
        if rays.shape[1] < 3:
            out.append((dbname, None, 0))
            continue
        P, inl = p3p_ransac(rays, X, np.radians(args.pnp_thr), args.ransac_iters, rng=rng)
        out.append((dbname, P, int(inl.sum())))
    return out


def _texture(Xw: np.ndarray) -> np.ndarray:
    """View-independent grey texture of a world point (0..255)."""
    t = np.sin(3.1 * Xw[:, 0]) + np.cos(4.3 * Xw[:, 1]) + np.sin(2.7 * Xw[:, 2] + Xw[:, 0])
    return (t + 3.0) / 6.0 * 255.0


def make_synthetic(root: str, n_queries: int, n_panos: int, rng):
    """Scene per query: a textured surface seen by a query camera.  Writes the
    shortlist, per-pano cutout XYZ maps, match files, the scan point clouds
    (+ identity transformations) and the query images.  Pano 0's matches are
    consistent with a WRONG pose (a plausible but false top-1 candidate), the
    other panos' with the true one, so dense pose verification has something
    to fix."""
    from scipy.io import savemat
    from PIL import Image
    import torch

    for d in ("cutouts/DUC1", "matches", "scans/DUC1/transformations", "queries"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    hq, wq, hd, wd, focal = 480, 640, 60, 80, 500.0
    Kq = np.array([[focal, 0, wq / 2.0], [0, focal, hq / 2.0], [0, 0, 1]])
    refs, shortlist = [], []
    for q in range(n_queries):
        A = rng.normal(size=(3, 3))
        R, _ = np.linalg.qr(A)
        R *= np.sign(np.linalg.det(R))
        t = rng.normal(size=3)
        P = np.hstack([R, t[:, None]])
        ang = np.radians(25.0)
        Rb = np.array([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]]) @ R
        P_bad = np.hstack([Rb, (t + np.array([1.5, 0.0, 0.5]))[:, None]])
        # dense textured surface covering the query view (camera frame), to world
        vv, uu = np.meshgrid(np.arange(0, hq, 1.5), np.arange(0, wq, 1.5), indexing="ij")
        z = 5.0 + 0.8 * np.sin(uu / 90.0) + 0.6 * np.cos(vv / 70.0)
        rays = np.linalg.solve(Kq, np.stack([uu.ravel(), vv.ravel(), np.ones(uu.size)]))
        Xc = (rays * z.ravel()).T
        Xw = (Xc - t) @ R
        gray = _texture(Xw)
        scan_id = f"{q:03d}"
        A_cell = np.empty((1, 7), dtype=object)
        for i, col in enumerate([Xw[:, 0], Xw[:, 1], Xw[:, 2], gray, gray, gray, gray]):
            A_cell[0, i] = col[:, None]
        savemat(os.path.join(root, "scans", "DUC1", f"DUC_scan_{scan_id}.ptx.mat"), {"A": A_cell})
        with open(os.path.join(root, "scans", "DUC1", "transformations", f"DUC_trans_{scan_id}.txt"), "w") as f:
            f.write("synthetic scan-to-global transform\n")
            f.write("\n".join(" ".join(f"{v:.1f}" for v in row) for row in np.eye(4)) + "\n")
        # query image: the scan rendered at the true pose
        img, _ = pv.points_to_perspective(torch.tensor(np.repeat(gray[:, None], 3, 1)), torch.tensor(Xw),
                                          torch.tensor(Kq @ P), hq, wq)
        g = pv.inpaint_nans(pv.rgb2gray(img)).clamp(0, 255).numpy().astype(np.uint8)
        Image.fromarray(np.repeat(g[..., None], 3, 2)).save(os.path.join(root, "queries", f"q{q}.jpg"), quality=95)
        names = []
        matches = np.zeros((1, n_panos, 400, 5))
        for p in range(n_panos):
            name = f"DUC1/{scan_id}/DUC_cutout_{scan_id}_{30 * p}_0"
            names.append(name)
            Pp = P_bad if p == 0 else P
            Rp, tp = Pp[:, :3], Pp[:, 3]
            # each cutout pixel stores a world point visible from the (claimed) camera
            Xcp = np.stack([rng.uniform(-2, 2, (hd, wd)), rng.uniform(-1.5, 1.5, (hd, wd)), rng.uniform(3, 9, (hd, wd))], -1)
            xyz = (Xcp - tp) @ Rp        # world = R^T (Xc - t), row-vector form
            os.makedirs(os.path.dirname(os.path.join(root, "cutouts", name)), exist_ok=True)
            savemat(os.path.join(root, "cutouts", name + ".mat"), {"XYZcut": xyz})
            n = 400
            rr, cc = rng.integers(0, hd - 1, n), rng.integers(0, wd - 1, n)
            # the reference looks up pixel floor(W*x) as a 1-based index: 0-based floor(W*x) - 1
            xd = np.stack([(cc + 1.5) / wd, (rr + 1.5) / hd], 1)
            pc = Xcp[rr, cc]
            xq = np.stack([(focal * pc[:, 0] / pc[:, 2] + wq / 2) / wq, (focal * pc[:, 1] / pc[:, 2] + hq / 2) / hq], 1)
            sc = np.full(n, 0.9)
            out = rng.random(n) < 0.3
            xq[out] = rng.random((out.sum(), 2))
            matches[0, p] = np.concatenate([xq, xd, sc[:, None]], 1)
        savemat(os.path.join(root, "matches", f"{q + 1}.mat"), {"matches": matches})
        refs.append({"queryname": f"q{q}.jpg", "P": P, "floor": "DUC1"})
        shortlist.append((f"q{q}.jpg", names))
    arr = np.empty((1, n_queries), dtype=[("queryname", "O"), ("topNname", "O")])
    for q, (qn, names) in enumerate(shortlist):
        arr[0, q] = (qn, np.array(names, dtype=object).reshape(1, -1))
    savemat(os.path.join(root, "shortlist.mat"), {"ImgList": arr})
    return refs, (hq, wq), focal


class ScanCache:
    """Loads each scan once (at_pv_wrapper.m groups candidates by scan)."""

    def __init__(self, scan_dir: str, suffix: str):
        self.scan_dir, self.suffix, self.cache = scan_dir, suffix, {}

    def get(self, dbname: str):
        scan_path, trans_path = pv.scan_paths(dbname, self.scan_dir, self.suffix)
        if scan_path not in self.cache:
            if not os.path.exists(scan_path):
                self.cache[scan_path] = None
            else:
                P_after = pv.load_transformation(trans_path) if os.path.exists(trans_path) else None
                self.cache[scan_path] = pv.load_scan(scan_path, P_after)
        return self.cache[scan_path]


def verify_query(qname: str, res, args, scans: ScanCache):
    """Dense-PV scores of one query's candidates, re-ranked (descending)."""
    from PIL import Image

    qpath = os.path.join(args.query_dir, qname)
    if not os.path.exists(qpath):
        return res, [0.0] * len(res)
    qimg = np.asarray(Image.open(qpath).convert("RGB"))
    scores = []
    for dbname, P, _ in res[: args.pv_topN]:
        scan = scans.get(dbname) if P is not None else None
        if scan is None:
            scores.append(0.0)
            continue
        s, _, _, _ = pv.pv_score(qimg, scan[0], scan[1], P, args.focal, device=args.pv_device)
        scores.append(float(s))
    ranked, sc = pv.rerank(res[: args.pv_topN], scores)
    return ranked, sc


def main(argv=None):
    ap = argparse.ArgumentParser(description="InLoc pose estimation from NC-Net matches")
    ap.add_argument("--matches_dir", type=str, default="")
    ap.add_argument("--shortlist", type=str, default="datasets/inloc/densePE_top100_shortlist_cvpr18.mat")
    ap.add_argument("--cutout_dir", type=str, default="datasets/inloc/cutouts")
    ap.add_argument("--trans_dir", type=str, default="")
    ap.add_argument("--query_size", type=int, nargs=2, default=[3024, 4032], help="query H W (iPhone7)")
    ap.add_argument("--focal", type=float, default=4032 * 28.0 / 36.0, help="query focal length in pixels")
    ap.add_argument("--pnp_topN", type=int, default=10)
    ap.add_argument("--thr", type=float, default=0.75)
    ap.add_argument("--pnp_thr", type=float, default=0.2, help="angular inlier threshold (degrees)")
    ap.add_argument("--n_subsample", type=int, default=None)
    ap.add_argument("--ransac_iters", type=int, default=10000)
    ap.add_argument("--rerank", choices=["none", "inliers"], default="none")
    ap.add_argument("--refposes", type=str, default="")
    ap.add_argument("--name", type=str, default="NCNet")
    ap.add_argument("--out", type=str, default="poses.npz")
    ap.add_argument("--pv", action="store_true", help="dense pose verification re-ranking of the top-N poses")
    ap.add_argument("--pv_topN", type=int, default=10)
    ap.add_argument("--scan_dir", type=str, default="datasets/inloc/scans")
    ap.add_argument("--scan_suffix", type=str, default=".ptx.mat")
    ap.add_argument("--query_dir", type=str, default="datasets/inloc/query/iphone7")
    ap.add_argument("--pv_device", type=str, default="cpu")
    ap.add_argument("--plot", type=str, default="", help="write the localization curves to this image")
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    rng = np.random.default_rng(args.seed)
    refs = None
    if args.synthetic:
        tmp = tempfile.mkdtemp(prefix="ncnet_loc_")
        refs, qsize, args.focal = make_synthetic(tmp, args.synthetic, 3, rng)
        args.query_size = list(qsize)
        args.matches_dir, args.shortlist = os.path.join(tmp, "matches"), os.path.join(tmp, "shortlist.mat")
        args.cutout_dir, args.pnp_topN = os.path.join(tmp, "cutouts"), 3
        args.scan_dir, args.query_dir = os.path.join(tmp, "scans"), os.path.join(tmp, "queries")
    queries, panos, _ = load_shortlist(args.shortlist)
    estimates, estimates_pv, records = {}, {}, []
    scans = ScanCache(args.scan_dir, args.scan_suffix) if args.pv else None
    for q, qname in enumerate(queries):
        mpath = os.path.join(args.matches_dir, f"{q + 1}.mat")
        if not os.path.exists(mpath):
            continue
        res = localize_query(_loadmat(mpath)["matches"], list(panos[q]), tuple(args.query_size), args, rng)
        pick = 0
        if args.rerank == "inliers":
            pick = int(np.argmax([r[2] for r in res]))
        estimates[qname] = (res[pick][0], res[pick][1])
        msg = f"{qname}: top-1 {res[pick][0]} inliers {res[pick][2]}"
        if args.pv:
            ranked, sc = verify_query(qname, res, args, scans)
            estimates_pv[qname] = (ranked[0][0], ranked[0][1])
            msg += f" | PV top-1 {ranked[0][0]} score {sc[0]:.3f}"
        records.append((qname, res))
        print(msg, flush=True)
    if records:
        np.savez(args.out, queries=np.array([r[0] for r in records]),
                 poses=np.array([[np.full((3, 4), np.nan) if p is None else p for _, p, _ in r[1]] for r in records]),
                 inliers=np.array([[n for _, _, n in r[1]] for r in records]))
    if args.refposes and refs is None:
        refs = load_refposes(args.refposes)
    rate = None
    if refs is not None:
        methods = [("DensePE + NCNet", "--b", estimates, args.name)]
        if args.pv:
            methods.append(("InLoc + NCNet", "--c", estimates_pv, args.name + "_PV"))
        curves = []
        for desc, marker, est, tag in methods:
            pos, ori = evaluate_queries(refs, est)
            r = localization_rate(pos, ori)
            with open(f"error_{tag}.txt", "w") as f:
                for ref, dp, do in zip(refs, pos, ori):
                    f.write(f"{ref['queryname']} {dp:f} {do:f}\n")
            print(desc)
            for thr, v in zip(DEFAULT_THRESHOLDS, r):
                print(f"  <{thr:.4f} m, <=10 deg: {100 * v:.1f}%")
            curves.append({"rate": r, "description": desc, "marker": marker})
        rate = curves[-1]["rate"] if args.pv else curves[0]["rate"]
        if args.plot:
            from ncnet_amd.utils.plot import plot_localization_curves
            plot_localization_curves(curves, args.plot)
    return (estimates_pv if args.pv else estimates), rate


if __name__ == "__main__":
    main()
