#!/usr/bin/env python
"""InLoc dense-match export (reference CLI: eval_inloc.py:29-40).

Writes ``matches/<folder>/<q+1>.mat`` with the reference's contract
(``matches`` [1, n_panos, N, 5], ``query_fn``, ``pano_fn``) for the MATLAB
localization pipeline.  Relocalization k=2 uses the fused correlation +
max-pool kernel (the full-resolution volume is never written).  Queries are
sharded over ranks (torchrun) and existing outputs are skipped (resume).

Extras: --synthetic_queries N builds a fake shortlist and random images in a
temp dir (smoke / benchmark without the dataset); --ncons_* for
checkpoint-less runs; --output_dir (default matches/); --precision
fp16|bf16|fp8|fp32 (default fp16, the reference's half_precision numerics:
bf16 trunk, IEEE-half features, correlation and NeighConsensus on the f16 MFMA;
bf16: bf16 operands; fp8: e4m3 correlation operands on the MX-fp8 MFMA with
the fused bf16 NeighConsensus; fp32: fp32 trunk + bf16x3 correlation and NC);
--fp8 = --precision fp8; --volume_parallel (under torchrun, every pair's
volume is sharded over all ranks instead of sharding the queries).
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.data.transforms import read_image  # noqa: E402
from ncnet_amd.engine.checkpoint import str_to_bool  # noqa: E402
from ncnet_amd.eval.inloc import (INLOC_CUDNN_BENCHMARK, PairMatcher, load_shortlist, n_matches, output_folder, pair_matches, prepare_image,  # noqa: E402
                                  save_query)
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.parallel.dist import barrier, destroy, init_distributed  # noqa: E402


def make_synthetic_inloc(root: str, n_queries: int, n_panos: int, h: int = 768, w: int = 1024):
    """Fake shortlist .mat + random JPEGs laid out like datasets/inloc."""
    from PIL import Image
    from scipy.io import savemat

    qdir, pdir = os.path.join(root, "query"), os.path.join(root, "pano")
    os.makedirs(qdir, exist_ok=True)
    os.makedirs(pdir, exist_ok=True)
    rng = np.random.default_rng(0)
    recs = []
    for q in range(n_queries):
        qn = f"IMG_{q:04d}.JPG"
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(os.path.join(qdir, qn))
        pn = []
        for p in range(n_panos):
            name = f"DUC1/pano_{q:03d}_{p:02d}.jpg"
            os.makedirs(os.path.dirname(os.path.join(pdir, name)), exist_ok=True)
            Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(os.path.join(pdir, name))
            pn.append(name)
        recs.append((qn, np.array(pn, dtype=object).reshape(1, -1)))
    arr = np.empty((1, n_queries), dtype=[("queryname", "O"), ("topNname", "O")])
    for q, (qn, pn) in enumerate(recs):
        arr[0, q] = (qn, pn)
    path = os.path.join(root, "synthetic_shortlist.mat")
    savemat(path, {"ImgList": arr})
    return path, qdir + "/", pdir + "/"


def _precision_kwargs(precision: str) -> dict:
    """--precision -> ImMatchNet (trunk dtype, correlation / NC operand dtype)."""
    return {"fp16": dict(dtype="bf16", corr_dtype="fp16"), "bf16": dict(dtype="bf16", corr_dtype="bf16"),
            "fp8": dict(dtype="bf16", corr_dtype="fp8"), "fp32": dict(dtype="fp32", corr_dtype="fp32")}[precision]


def main(argv=None):
    ap = argparse.ArgumentParser(description="Compute InLoc matches")
    ap.add_argument("--checkpoint", type=str, default="")
    ap.add_argument("--inloc_shortlist", type=str, default="datasets/inloc/densePE_top100_shortlist_cvpr18.mat")
    ap.add_argument("--k_size", type=int, default=2)
    ap.add_argument("--image_size", type=int, default=3200)
    ap.add_argument("--n_queries", type=int, default=356)
    ap.add_argument("--n_panos", type=int, default=10)
    ap.add_argument("--softmax", type=str_to_bool, default=True)
    ap.add_argument("--matching_both_directions", type=str_to_bool, default=True)
    ap.add_argument("--flip_matching_direction", type=str_to_bool, default=False)
    ap.add_argument("--pano_path", type=str, default="datasets/inloc/pano/")
    ap.add_argument("--query_path", type=str, default="datasets/inloc/query/iphone7/")
    ap.add_argument("--output_dir", type=str, default="matches/")
    ap.add_argument("--synthetic_queries", type=int, default=0)
    ap.add_argument("--synthetic_hw", type=int, nargs=2, default=[768, 1024],
                    help="height width of the --synthetic_queries images (default 768 1024, 4:3 landscape)")
    ap.add_argument("--ncons_kernel_sizes", nargs="+", type=int, default=[3, 3])
    ap.add_argument("--ncons_channels", nargs="+", type=int, default=[16, 1])
    ap.add_argument("--precision", choices=["fp16", "bf16", "fp8", "fp32"], default="fp16",
                    help="fp16 (default; the reference's half precision on the f16 MFMA), bf16, fp8 (e4m3 "
                         "correlation operands, fused bf16 NeighConsensus), fp32 (fp32 trunk, bf16x3 correlation + NC)")
    ap.add_argument("--fp8", action="store_true",
                    help="= --precision fp8: OCP e4m3 correlation operands on the MX-fp8 MFMA; the NeighConsensus "
                         "stays on the fused bf16 kernel (measured faster; NCNET_NC_FP8=1 selects the fp8 Conv4d "
                         "kernels)")
    ap.add_argument("--volume_parallel", action="store_true",
                    help="all ranks cooperate on every pair, sharding its 4D volume along the A rows "
                         "(ncnet_amd/parallel/volume_parallel.py); default: queries sharded over ranks")
    args = ap.parse_args(argv)
    ctx = init_distributed()

    tmp = None
    if args.synthetic_queries:
        tmp = tempfile.mkdtemp(prefix="ncnet_inloc_")
        args.inloc_shortlist, args.query_path, args.pano_path = make_synthetic_inloc(
            tmp, args.synthetic_queries, args.n_panos, *args.synthetic_hw)
        args.n_queries = args.synthetic_queries
    torch.backends.cudnn.benchmark = INLOC_CUDNN_BENCHMARK   # the state bench.py's InLoc secondaries time
    torch.manual_seed(1)   # checkpoint-less (synthetic) runs: the same random NC weights on every launch
    model = ImMatchNet(use_cuda=ctx.device.type == "cuda", checkpoint=args.checkpoint or None,
                       ncons_kernel_sizes=args.ncons_kernel_sizes, ncons_channels=args.ncons_channels,
                       half_precision=True, relocalization_k_size=args.k_size,
                       **_precision_kwargs("fp8" if args.fp8 else args.precision)).to(ctx.device)
    model.eval()
    vp = None
    if args.volume_parallel and ctx.world_size > 1:
        from ncnet_amd.parallel.dist import broadcast_module
        from ncnet_amd.parallel.volume_parallel import VolumeParallelMatcher
        broadcast_module(model, ctx)
        vp = VolumeParallelMatcher(model, ctx)
    q_start, q_step = (0, 1) if vp is not None else (ctx.rank, ctx.world_size)
    folder = output_folder(args.inloc_shortlist, args.image_size, args.k_size, args.matching_both_directions,
                           args.flip_matching_direction, args.softmax, args.checkpoint)
    out_dir = os.path.join(args.output_dir, folder)
    os.makedirs(out_dir, exist_ok=True)
    if ctx.is_main:
        print("Output matches folder: " + folder)
    queries, panos, pano_all = load_shortlist(args.inloc_shortlist)
    matcher = PairMatcher(model, args.k_size, args.softmax, args.matching_both_directions,
                          args.flip_matching_direction)
    N = n_matches(args.image_size, args.k_size, args.matching_both_directions)
    nq = min(args.n_queries, len(queries))
    t0 = time.perf_counter()
    npairs = 0
    with torch.inference_mode():
        for q in range(q_start, nq, q_step):
            path = os.path.join(out_dir, f"{q + 1}.mat")
            if os.path.exists(path):
                continue
            src = prepare_image(read_image(os.path.join(args.query_path, queries[q])), args.image_size, args.k_size,
                                ctx.device)
            npq = min(args.n_panos, len(panos[q]))
            tgts = [prepare_image(read_image(os.path.join(args.pano_path, panos[q][idx])), args.image_size,
                                  args.k_size, ctx.device) for idx in range(npq)]
            if vp is None:
                # the query's features are extracted once for its n_panos pairs and
                # the panos' trunk runs as one batch when their sizes agree (the
                # reference re-runs both backbones per pair; identical features)
                if all(t.shape == src.shape for t in tgts):
                    # query and panos in one trunk batch (InLoc resizes both to the same size)
                    fb_, hwp = model.extract(torch.cat([src] + tgts, 0))
                    sl = lambda i: tuple(t[i:i + 1] for t in fb_) if isinstance(fb_, tuple) else fb_[i:i + 1]  # noqa: E731
                    fq = (sl(0), hwp)
                    fps = [(sl(i + 1), hwp) for i in range(npq)]
                elif npq > 1 and all(t.shape == tgts[0].shape for t in tgts):
                    fq = model.extract(src)
                    fpb, hwp = model.extract(torch.cat(tgts, 0))
                    fps = [(tuple(t[i:i + 1] for t in fpb) if isinstance(fpb, tuple) else fpb[i:i + 1], hwp)
                           for i in range(npq)]
                else:
                    fq = model.extract(src)
                    fps = [model.extract(t) for t in tgts]
            pair_ms = []
            for idx in range(npq):
                if vp is not None:
                    out = vp.forward({"source_image": src, "target_image": tgts[idx]})
                    corr4d, delta4d = out if args.k_size > 1 else (out, None)
                    m = pair_matches(corr4d, delta4d, args.k_size, args.softmax, args.matching_both_directions,
                                     args.flip_matching_direction).double().cpu().numpy()
                else:
                    # correlation .. match extraction as one HIP graph per shape
                    res, cnt = matcher(fq[0], fq[1], fps[idx][0], fps[idx][1])
                    m = res[:int(cnt)].double().cpu().numpy()
                pair_ms.append(m)
                npairs += 1
            # the reference's N (eval_inloc.py:116-118) is sized for 4:3 landscape
            # images; a pair with more unique matches (square / other aspect ratios)
            # grows the array instead of being truncated -- the MATLAB side squeezes
            # it, so the row count is free -- and the reference itself would fail
            # on the overflow (eval_inloc.py:197-203), never drop rows silently
            nq_rows = max([N] + [len(m) for m in pair_ms])
            if nq_rows > N:
                print(f"query {q + 1}: {nq_rows} matches exceed N={N} (4:3 sizing); "
                      f"writing {nq_rows} rows", file=sys.stderr, flush=True)
            matches = np.zeros((1, args.n_panos, nq_rows, 5))
            for idx, m in enumerate(pair_ms):
                matches[0, idx, :len(m)] = m
            if vp is None or ctx.is_main:
                save_query(path, matches, queries[q], pano_all)
            if ctx.is_main:
                print(f"query {q + 1}/{nq} ({npairs} pairs, {npairs / (time.perf_counter() - t0):.2f} pairs/s/rank)",
                      flush=True)
    barrier(ctx)
    if ctx.is_main:
        print("Done: " + out_dir)
    destroy(ctx)
    return out_dir


if __name__ == "__main__":
    main()
