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

Every (query, cutout) pair is an independent task with its own seeded
generator, run on --workers spawned processes (the reference's parfor over
queries, ir_top100_NC4D_localization_pnponly.m:25, and over unique scans for
PV, ht_top10_NC4D_PV_localization.m:44); results do not depend on the worker
count.  --cache_dir keeps one file per pair (parfor_NC4D_PE_pnponly.m:4-6
skips pairs whose .mat exists), so an interrupted run resumes.

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


def _pair_rng(seed: int, q: int, jj: int):
    """Per-(query, cutout) generator: results do not depend on the worker count
    or the order the pairs run in."""
    return np.random.default_rng([seed, q, jj])


def _cache_path(cache_dir: str, qname: str, dbname: str, kind: str) -> str:
    """parfor_NC4D_PE_pnponly.m:4 / parfor_nc4d_PV.m: one file per (query, db).
    The full relative cutout name keeps same-named cutouts of different scans
    apart."""
    rel = os.path.normpath(dbname).lstrip(os.sep)
    if rel.startswith(".."):
        raise ValueError(f"cutout name escapes the cache dir: {dbname!r}")
    return os.path.join(cache_dir, kind, qname, rel + ".npz")


_PNP_KEYS = ("thr", "pnp_thr", "ransac_iters", "n_subsample", "seed", "focal")


def _cache_key(cfg: dict, keys, *arrays, extra=()) -> str:
    """Hash of everything a cached result depends on: the run settings named in
    ``keys``, the pair's inputs (its match rows, the scored pose P) and
    ``extra``.  A cached file whose key differs is recomputed, never reused."""
    import hashlib
    h = hashlib.sha256()
    h.update(repr([(k, cfg[k]) for k in keys] + list(extra)).encode())
    for a in arrays:
        if a is None:
            h.update(b"<none>")
        else:
            a = np.ascontiguousarray(np.asarray(a, np.float64))
            h.update(repr(a.shape).encode())
            h.update(a.tobytes())
    return h.hexdigest()


def _cache_load(cpath, key):
    """The cached npz when it exists and was written under ``key``, else None."""
    if not cpath or not os.path.exists(cpath):
        return None
    z = np.load(cpath)   # plain arrays only (allow_pickle stays False)
    if "key" not in z.files or str(z["key"]) != key:
        return None
    return z


def _pnp_pair(task):
    """One (query, cutout) pair: threshold, tentatives, P3P LO-RANSAC
    (parfor_NC4D_PE_pnponly.m).  Cached on disk when cache_dir is set."""
    q, jj, qname, dbname, m, q_size, cfg = task
    cpath = _cache_path(cfg["cache_dir"], qname, dbname, "pnp") if cfg["cache_dir"] else None
    key = _cache_key(cfg, _PNP_KEYS, m, extra=(tuple(q_size), q, jj)) if cpath else ""
    z = _cache_load(cpath, key)
    if z is not None:
        P = z["P"]
        return q, jj, dbname, (None if np.isnan(P).all() else P), int(z["n_inliers"])
    P, n_inl = None, 0
    xyz_path = os.path.join(cfg["cutout_dir"], dbname + ".mat")
    if m is not None and os.path.exists(xyz_path):
        xyz = _loadmat(xyz_path)["XYZcut"].astype(np.float64)
        P_after = None
        if cfg["trans_dir"]:
            tp = os.path.join(cfg["trans_dir"], dbname + ".txt")
            if os.path.exists(tp):
                P_after = np.loadtxt(tp)
        rng = _pair_rng(cfg["seed"], q, jj)
        rays, X, _, _ = tentative_correspondences(m, cfg["thr"], q_size, xyz, cfg["focal"], P_after,
                                                  cfg["n_subsample"], rng)
        if rays.shape[1] >= 3:
            P, inl = p3p_ransac(rays, X, np.radians(cfg["pnp_thr"]), cfg["ransac_iters"], rng=rng)
            n_inl = int(inl.sum())
    if cpath:
        os.makedirs(os.path.dirname(cpath), exist_ok=True)
        tmp = cpath + ".tmp.npz"
        np.savez(tmp, P=np.full((3, 4), np.nan) if P is None else P, n_inliers=n_inl, key=key)
        os.replace(tmp, cpath)
    return q, jj, dbname, P, n_inl


def _cfg(args) -> dict:
    return {k: getattr(args, k) for k in ("cutout_dir", "trans_dir", "thr", "focal", "n_subsample", "pnp_thr",
                                          "ransac_iters", "seed", "cache_dir", "query_dir", "pv_device")}


def localize_query(q_matches: np.ndarray, db_names, q_size, args, q: int = 0, qname: str = "query"):
    """q_matches [1, n_panos, N, 5] -> list of (dbname, P or None, n_inliers), serially."""
    cfg = _cfg(args)
    out = []
    for jj, dbname in enumerate(db_names[: args.pnp_topN]):
        m = q_matches[0, jj] if jj < q_matches.shape[1] else None
        _, _, name, P, n = _pnp_pair((q, jj, qname, dbname, m, q_size, cfg))
        out.append((name, P, n))
    return out


def _executor(workers: int):
    """Spawned worker processes (the parent may hold OpenMP / torch threads that
    do not survive a fork); MATLAB's parpool in the reference."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    return ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn"),
                               initializer=_worker_init)


def _worker_init():
    try:
        import torch
        torch.set_num_threads(1)
    except Exception:  # pragma: no cover
        pass


def localize_all(jobs, args):
    """jobs: [(q, qname, matches [1, n_panos, N, 5], db_names)] -> {q: [(dbname, P, n_inl)] * topN}.
    Every (query, cutout) pair is one task (ir_top100_NC4D_localization_pnponly.m:25
    parfors over queries; pairs balance better when queries have few panos)."""
    cfg, q_size = _cfg(args), tuple(args.query_size)
    tasks = []
    for q, qname, mats, names in jobs:
        for jj, dbname in enumerate(list(names)[: args.pnp_topN]):
            m = mats[0, jj] if jj < mats.shape[1] else None
            tasks.append((q, jj, qname, dbname, m, q_size, cfg))
    res = {q: [None] * min(len(names), args.pnp_topN) for q, _, _, names in jobs}
    if args.workers > 1 and len(tasks) > 1:
        with _executor(args.workers) as ex:
            outs = list(ex.map(_pnp_pair, tasks, chunksize=max(1, len(tasks) // (4 * args.workers))))
    else:
        outs = [_pnp_pair(t) for t in tasks]
    for q, jj, dbname, P, n in outs:
        res[q][jj] = (dbname, P, n)
    return res


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


def _pv_scan(task):
    """All candidates that render from one scan (at_pv_wrapper.m: load the scan
    once, then parfor_nc4d_PV.m per (query, cutout, P)).  Returns
    [(q, jj, score)]; scores are cached per pair when cache_dir is set."""
    scan_path, trans_path, items, cfg = task
    from PIL import Image
    out, todo = [], []
    for q, jj, qname, dbname, P in items:
        cpath = _cache_path(cfg["cache_dir"], qname, dbname, "pv") if cfg["cache_dir"] else None
        key = _cache_key(cfg, ("focal",), P, extra=(os.path.basename(scan_path),)) if cpath else ""
        z = _cache_load(cpath, key)
        if z is not None:
            out.append((q, jj, float(z["score"])))
        else:
            todo.append((q, jj, qname, dbname, P, cpath, key))
    if not todo:
        return out
    scan = None
    if os.path.exists(scan_path):
        P_after = pv.load_transformation(trans_path) if os.path.exists(trans_path) else None
        scan = pv.load_scan(scan_path, P_after)
    qimgs = {}
    for q, jj, qname, dbname, P, cpath, key in todo:
        qpath = os.path.join(cfg["query_dir"], qname)
        s = 0.0
        if scan is not None and P is not None and os.path.exists(qpath):
            if qname not in qimgs:
                qimgs[qname] = np.asarray(Image.open(qpath).convert("RGB"))
            s = float(pv.pv_score(qimgs[qname], scan[0], scan[1], P, cfg["focal"], device=cfg["pv_device"])[0])
        if cpath:
            os.makedirs(os.path.dirname(cpath), exist_ok=True)
            tmp = cpath + ".tmp.npz"
            np.savez(tmp, score=s, key=key)
            os.replace(tmp, cpath)
        out.append((q, jj, s))
    return out


def verify_all(results, qnames, args):
    """Dense pose verification of every query's top-N candidates, grouped by
    scan (ht_top10_NC4D_PV_localization.m:30-47), then the per-query re-rank.
    results: {q: [(dbname, P, n)]} -> {q: (ranked candidates, scores)}."""
    cfg = _cfg(args)
    groups = {}
    for q, res in results.items():
        for jj, (dbname, P, _) in enumerate(res[: args.pv_topN]):
            scan_path, trans_path = pv.scan_paths(dbname, args.scan_dir, args.scan_suffix)
            groups.setdefault((scan_path, trans_path), []).append((q, jj, qnames[q], dbname, P))
    tasks = [(sp, tp, items, cfg) for (sp, tp), items in sorted(groups.items())]
    if args.workers > 1 and len(tasks) > 1 and args.pv_device == "cpu":
        with _executor(args.workers) as ex:
            outs = [o for part in ex.map(_pv_scan, tasks) for o in part]
    else:
        outs = [o for t in tasks for o in _pv_scan(t)]
    scores = {q: [0.0] * min(len(res), args.pv_topN) for q, res in results.items()}
    for q, jj, s in outs:
        scores[q][jj] = s
    return {q: pv.rerank(results[q][: args.pv_topN], scores[q]) for q in results}


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
    ap.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1),
                    help="worker processes for the per-pair P3P RANSAC and the per-scan PV (1 = serial)")
    ap.add_argument("--cache_dir", type=str, default="",
                    help="per-(query, cutout) result cache (pnp/<query>/<db>.npz, pv/...); reruns skip cached pairs")
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
    jobs = []
    for q, qname in enumerate(queries):
        mpath = os.path.join(args.matches_dir, f"{q + 1}.mat")
        if os.path.exists(mpath):
            jobs.append((q, qname, _loadmat(mpath)["matches"], list(panos[q])))
    results = localize_all(jobs, args)
    qnames = {q: qname for q, qname, _, _ in jobs}
    verified = verify_all(results, qnames, args) if args.pv else {}
    for q, qname, _, _ in jobs:
        res = results[q]
        pick = 0
        if args.rerank == "inliers":
            pick = int(np.argmax([r[2] for r in res]))
        estimates[qname] = (res[pick][0], res[pick][1])
        msg = f"{qname}: top-1 {res[pick][0]} inliers {res[pick][2]}"
        if args.pv:
            ranked, sc = verified[q]
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
