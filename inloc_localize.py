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

Inputs on disk (InLoc layout): --cutout_dir/<dbname>.mat with 'XYZcut'
[H,W,3]; optional --trans_dir/<dbname>.txt holding the 4x4 (or 3x4)
scan-to-global matrix.  --synthetic N builds a fake scene to smoke-test the
whole chain.  Dense pose verification (synthetic-view rendering) is out of scope.
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


def make_synthetic(root: str, n_queries: int, n_panos: int, rng):
    """Scene: random 3D points seen by a query camera; cutout XYZ maps and
    matches consistent with the true query pose (plus outliers)."""
    from scipy.io import savemat

    os.makedirs(os.path.join(root, "cutouts", "DUC1"), exist_ok=True)
    os.makedirs(os.path.join(root, "matches"), exist_ok=True)
    hq, wq, hd, wd, focal = 480, 640, 60, 80, 500.0
    refs, shortlist = [], []
    for q in range(n_queries):
        A = rng.normal(size=(3, 3))
        R, _ = np.linalg.qr(A)
        R *= np.sign(np.linalg.det(R))
        t = rng.normal(size=3)
        P = np.hstack([R, t[:, None]])
        names = []
        matches = np.zeros((1, n_panos, 400, 5))
        for p in range(n_panos):
            name = f"DUC1/cut_{q:03d}_{p:02d}"
            names.append(name)
            # each cutout pixel stores a world point visible from the query camera
            Xc = np.stack([rng.uniform(-2, 2, (hd, wd)), rng.uniform(-1.5, 1.5, (hd, wd)), rng.uniform(3, 9, (hd, wd))], -1)
            xyz = (Xc - t) @ R        # world = R^T (Xc - t), row-vector form
            savemat(os.path.join(root, "cutouts", name + ".mat"), {"XYZcut": xyz})
            n = 400
            rr, cc = rng.integers(0, hd - 1, n), rng.integers(0, wd - 1, n)
            # the reference looks up pixel floor(W*x) as a 1-based index: 0-based floor(W*x) - 1
            xd = np.stack([(cc + 1.5) / wd, (rr + 1.5) / hd], 1)
            pc = Xc[rr, cc]
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
    queries, panos, _ = load_shortlist(args.shortlist)
    estimates, records = {}, []
    for q, qname in enumerate(queries):
        mpath = os.path.join(args.matches_dir, f"{q + 1}.mat")
        if not os.path.exists(mpath):
            continue
        res = localize_query(_loadmat(mpath)["matches"], list(panos[q]), tuple(args.query_size), args, rng)
        pick = 0
        if args.rerank == "inliers":
            pick = int(np.argmax([r[2] for r in res]))
        estimates[qname] = (res[pick][0], res[pick][1])
        records.append((qname, res))
        print(f"{qname}: top-1 {res[pick][0]} inliers {res[pick][2]}", flush=True)
    if records:
        np.savez(args.out, queries=np.array([r[0] for r in records]),
                 poses=np.array([[np.full((3, 4), np.nan) if p is None else p for _, p, _ in r[1]] for r in records]),
                 inliers=np.array([[n for _, _, n in r[1]] for r in records]))
    if args.refposes and refs is None:
        refs = load_refposes(args.refposes)
    rate = None
    if refs is not None:
        pos, ori = evaluate_queries(refs, estimates)
        rate = localization_rate(pos, ori)
        with open(f"error_{args.name}.txt", "w") as f:
            for r, dp, do in zip(refs, pos, ori):
                f.write(f"{r['queryname']} {dp:f} {do:f}\n")
        for thr, v in zip(DEFAULT_THRESHOLDS, rate):
            print(f"  <{thr:.4f} m, <=10 deg: {100 * v:.1f}%")
    return estimates, rate


if __name__ == "__main__":
    main()
