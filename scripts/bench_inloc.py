#!/usr/bin/env python
"""InLoc dense-matching inference benchmark (BASELINE configs 4 and 5).

One query/pano pair per forward, exactly the eval_inloc.py hot path
(reference eval_inloc.py:124-189): backbone on both images, fused
correlation + 2x2x2x2 max-pool (relocalization k=2), MutualMatching,
NeighConsensus (3,3 / 16,1), MutualMatching, then bidirectional match
extraction with GPU de-duplication.  Synthetic 4:3 images (random pixels,
random-init weights); the images are resized exactly like eval_inloc
(longest side -> --image-size, floored to a multiple of 32 px).

Prints one JSON line with ms/pair and a per-stage breakdown (CUDA events).

    python scripts/bench_inloc.py --image-size 1600 --pairs 5 --warmup 2
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/bench_inloc.py --image-size 3200 --fp8 --volume-parallel

--volume-parallel: every pair's volume is sharded along its A rows over all
ranks (ncnet_amd/parallel/volume_parallel.py); the latency is the max over
ranks and includes the final gather of the volume (no per-stage breakdown).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from ncnet_amd import config as _config  # noqa: E402
from ncnet_amd.eval.inloc import n_matches, pair_matches, target_size  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.ops.correlation import correlation, correlation_pool2  # noqa: E402


def run_single(image_size: int = 1600, fp8: bool = False, pairs: int = 5, warmup: int = 2, k: int = 2,
               ncons_kernel_sizes=(3, 3), ncons_channels=(16, 1), src_hw=(3024, 4032), no_matches: bool = False,
               impl: str = "hip", model=None, panos_per_query: int = 1, pair_graph: bool | None = None,
               precision: str | None = None) -> dict:
    """One InLoc query/pano pair per forward on one GPU; returns the JSON record.

    panos_per_query > 1: eval_inloc.py's schedule -- the query's features are
    extracted once and reused for that many consecutive pairs, and the panos'
    trunk runs as one batch (the reference runs both backbones per pair; the
    matches are identical), so ``pairs`` should be a multiple of it.  1: both
    backbones per pair.  pair_graph (default: with panos_per_query > 1, as
    eval_inloc.py does): everything after the backbones replayed as one HIP
    graph (eval/inloc.py PairMatcher); its time is reported as "pair_graph",
    and an untimed eager pass afterwards gives the per-stage breakdown
    ("stages_ms_eager": corr_pool, mm_nc_mm, matches)."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # precision: bf16 (bf16 trunk + operands), fp16 (bf16 trunk, IEEE-half
    # features / correlation / NC: the reference's half_precision numerics on the
    # f16 MFMA), fp8 (bf16 trunk, e4m3 correlation operands)
    precision = precision or ("fp8" if fp8 else "bf16")
    if model is None:
        model = ImMatchNet(use_cuda=True, ncons_kernel_sizes=list(ncons_kernel_sizes),
                           ncons_channels=list(ncons_channels), half_precision=True, relocalization_k_size=k,
                           corr_dtype=precision).to(dev).eval()
    model.corr_dtype = precision
    model.compute_dtype = torch.bfloat16     # the trunk (fp16: halved after the L2 norm, as the reference)
    fp8 = precision == "fp8"
    h, w = target_size(src_hw[0], src_hw[1], image_size, k)
    if pair_graph is None:
        pair_graph = panos_per_query > 1 and _config.RUNTIME.pair_graph
    src = torch.randn(1, 3, h, w, device=dev)
    tgt = torch.randn(1, 3, h, w, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    stages = {"backbone": 0.0, "corr_pool": 0.0, "mm_nc_mm": 0.0, "matches": 0.0}
    if pair_graph:
        stages = {"backbone": 0.0, "pair_graph": 0.0}
    nmatch = 0
    eager_stages = False

    if impl == "reference":
        from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_inloc_forward
        alg = ReferenceAlgorithm(model, torch.float32)

    def one_ref(timed: bool):
        nonlocal nmatch
        with torch.inference_mode():
            ev[0].record()
            corr4d, delta = reference_inloc_forward(alg, src, tgt, k)
            ev[3].record()
            if not no_matches:
                m = pair_matches(corr4d.float(), tuple(d.long() for d in delta) if delta else None, k, True, True)
                nmatch = int(m.shape[0])
            ev[4].record()
        if timed:
            torch.cuda.synchronize()
            stages["mm_nc_mm"] += ev[0].elapsed_time(ev[3])
            stages["matches"] += ev[3].elapsed_time(ev[4])

    fq = None
    fpano = {}
    from ncnet_amd.eval.inloc import PairMatcher
    matcher = PairMatcher(model, k) if pair_graph else None

    def one(timed: bool, new_query: bool = True):
        if impl == "reference":
            return one_ref(timed)
        nonlocal nmatch, fq
        with torch.inference_mode():
            ev[0].record()
            if panos_per_query <= 1:
                f, (fh, fw) = model.extract(torch.cat((src, tgt), 0))
                fa, fb = f[:1], f[1:]
            else:
                # eval_inloc.py: the query's features are extracted once for its
                # panos, and the panos' trunk runs as one batch
                if new_query or fq is None:
                    # the query and its panos in one trunk batch (eval_inloc.py)
                    fall, hw_ = model.extract(torch.cat((src, tgt.expand(panos_per_query, -1, -1, -1)), 0))
                    fq = (fall[:1], hw_)
                    fpano["f"] = fall[1:]
                    fpano["i"] = 0
                fa, (fh, fw) = fq
                fb = fpano["f"][fpano["i"]:fpano["i"] + 1]
                fpano["i"] += 1
            ev[1].record()
            if matcher is not None and not eager_stages:
                # correlation .. match extraction replayed as one HIP graph (eval_inloc.py)
                res, cnt = matcher(fa, (fh, fw), fb, (fh, fw))
                ev[2].record()
                if timed:
                    nmatch = int(cnt)
                    torch.cuda.synchronize()
                    stages["backbone"] += ev[0].elapsed_time(ev[1])
                    stages["pair_graph"] += ev[1].elapsed_time(ev[2])
                return
            if k == 2:
                corr4d, delta = correlation_pool2(fa, fb, fh, fw, fh, fw)
            else:
                corr4d, delta = correlation(fa, fb).view(1, 1, fh, fw, fh, fw), None
            ev[2].record()
            corr4d = model.process_correlation(corr4d)
            ev[3].record()
            if not no_matches:
                m = pair_matches(corr4d, delta, k, True, True)
                nmatch = int(m.shape[0])
            ev[4].record()
        if timed:
            torch.cuda.synchronize()
            for i, kk in enumerate(stages):
                stages[kk] += ev[i].elapsed_time(ev[i + 1])

    for i in range(warmup):
        one(False, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(pairs):
        one(True, i % max(1, panos_per_query) == 0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / pairs
    timed_stages = {kk: round(v / pairs, 3) for kk, v in stages.items()}
    eager = None
    if matcher is not None and impl != "reference":
        # the graph replays correlation .. matches as one unit: break it down
        # with an untimed eager pass over the same pairs (same kernels, with
        # the launch gaps the graph removes)
        eager_stages = True
        # warm the eager path first (its own allocations, first-call kernel
        # loads and host-side caches are not the graph's): untimed passes,
        # then the timed breakdown
        for i in range(2):
            one(False, i == 0)
        torch.cuda.synchronize()
        stages = {"backbone": 0.0, "corr_pool": 0.0, "mm_nc_mm": 0.0, "matches": 0.0}
        n_eager = max(3, min(pairs, 5))
        for i in range(n_eager):
            one(True, i == 0)
        eager = {kk: round(v / n_eager, 3) for kk, v in stages.items() if kk != "backbone"}
    fs = (h // 16 // k, w // 16 // k)
    return {
        "metric": "InLoc dense matching latency per pair (fwd, k=%d relocalization)" % k,
        "value": round(ms, 3), "unit": "ms/pair", "higher_is_better": False,
        "pairs_per_s": round(1e3 / ms, 3), "n_gpus": 1, "pairs": pairs, "warmup": warmup,
        "impl": impl,
        "dtype": ("fp32-backbone/fp16-volume" if impl == "reference" else
                  (("fp8-corr+fp8-nc" if _config.RUNTIME.nc_fp8 else "fp8-corr+bf16-fused-nc")
                   if fp8 else precision)),
        "data": "synthetic (random 4:3 images, random-init weights)",
        "config": {"image": [h, w], "features": [h // 16, w // 16], "volume": list(fs) * 2,
                   "ncons": [list(ncons_kernel_sizes), list(ncons_channels)], "k": k,
                   "panos_per_query": panos_per_query},
        "stages_ms": timed_stages,
        **({"stages_ms_eager": eager} if eager is not None else {}),
        "matches": nmatch, "matches_contract": n_matches(image_size, k, True),
        # loud: the record says whether the pair graph actually replayed
        "pair_graph": bool(matcher is not None and matcher.graphed),
        **({"pair_graph_error": matcher.capture_error.strip().splitlines()[-1][:300]}
           if matcher is not None and matcher.capture_error else {}),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image-size", type=int, default=1600)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ncons_kernel_sizes", nargs="+", type=int, default=[3, 3])
    ap.add_argument("--ncons_channels", nargs="+", type=int, default=[16, 1])
    ap.add_argument("--src-hw", type=int, nargs=2, default=[3024, 4032], help="raw query size (iPhone7)")
    ap.add_argument("--no-matches", action="store_true")
    ap.add_argument("--panos-per-query", type=int, default=1,
                    help="eval_inloc.py schedule: query features extracted once per this many pairs (10 in InLoc)")
    ap.add_argument("--fp8", action="store_true",
                    help="OCP e4m3 correlation operands (MX-fp8 MFMA); the NC runs the fused bf16 kernel "
                         "(NCNET_NC_FP8=1: the fp8 Conv4d kernels instead)")
    ap.add_argument("--precision", choices=["bf16", "fp16", "fp8"], default=None,
                    help="operand precision (default bf16, or fp8 with --fp8); fp16 = the reference's half "
                         "precision on the f16 MFMA")
    ap.add_argument("--impl", choices=["hip", "reference"], default="hip",
                    help="reference: the reference algorithm in plain PyTorch-ROCm (fp32 backbone, fp16 volume)")
    ap.add_argument("--volume-parallel", action="store_true")
    a = ap.parse_args()
    if a.volume_parallel:
        return bench_volume_parallel(a)
    print(json.dumps(run_single(a.image_size, a.fp8, a.pairs, a.warmup, a.k, a.ncons_kernel_sizes, a.ncons_channels,
                                a.src_hw, a.no_matches, a.impl, panos_per_query=a.panos_per_query,
                                precision=a.precision)))


def bench_volume_parallel(a):
    from ncnet_amd.parallel.dist import all_reduce_max_float, barrier, broadcast_module, destroy, init_distributed
    from ncnet_amd.parallel.volume_parallel import VolumeParallelMatcher

    ctx = init_distributed()
    dev = ctx.device
    torch.manual_seed(0)
    model = ImMatchNet(use_cuda=dev.type == "cuda", ncons_kernel_sizes=a.ncons_kernel_sizes,
                       ncons_channels=a.ncons_channels, half_precision=True, relocalization_k_size=a.k,
                       corr_dtype="fp8" if a.fp8 else "bf16").to(dev).eval()
    broadcast_module(model, ctx)
    vp = VolumeParallelMatcher(model, ctx)
    h, w = target_size(a.src_hw[0], a.src_hw[1], a.image_size, a.k)
    g = torch.Generator(device=dev).manual_seed(0)
    batch = {"source_image": torch.randn(1, 3, h, w, device=dev, generator=g),
             "target_image": torch.randn(1, 3, h, w, device=dev, generator=g)}
    nmatch = 0

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def one():
        nonlocal nmatch
        with torch.inference_mode():
            out = vp.forward(batch)
            corr4d, delta = out if a.k > 1 else (out, None)
            if not a.no_matches and ctx.is_main:
                nmatch = int(pair_matches(corr4d, delta, a.k, True, True).shape[0])

    for _ in range(a.warmup):
        one()
    sync()
    barrier(ctx)
    t0 = time.perf_counter()
    for _ in range(a.pairs):
        one()
    sync()
    barrier(ctx)
    ms = all_reduce_max_float((time.perf_counter() - t0) * 1e3 / a.pairs, ctx)
    if ctx.is_main:
        fs = (h // 16 // a.k, w // 16 // a.k)
        print(json.dumps({
            "metric": "InLoc dense matching latency per pair (fwd, k=%d relocalization, volume parallel)" % a.k,
            "value": round(ms, 3), "unit": "ms/pair", "higher_is_better": False, "pairs_per_s": round(1e3 / ms, 3),
            "n_gpus": ctx.world_size, "pairs": a.pairs, "warmup": a.warmup, "impl": "hip",
            "dtype": "fp8-corr/bf16" if a.fp8 else "bf16", "data": "synthetic (random 4:3 images, random-init weights)",
            "config": {"image": [h, w], "volume": list(fs) * 2, "ncons": [a.ncons_kernel_sizes, a.ncons_channels],
                       "k": a.k, "parallelism": f"vp{ctx.world_size}"},
            "matches": nmatch}))
    destroy(ctx)


if __name__ == "__main__":
    main()
