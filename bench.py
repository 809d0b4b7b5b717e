#!/usr/bin/env python
"""Headline benchmark: image-pairs/s, fwd+bwd training step of ResNet-101 +
NC-Net (5,5,5 / 16,16,1) at 400x400, bf16, synthetic pairs, random init
(BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--impl hip|reference]

One process per GPU (torchrun env for N > 1; RCCL all-reduce of gradients).
A step is exactly what train.py does per batch: zero_grad, backbone on the
pair images (queued one step ahead on a side stream while the frozen trunk
allows it: engine/trainer.py TrunkPrefetcher), correlation of positive and rolled-negative pairs, MutualMatching,
symmetric NeighConsensus, MutualMatching, weak loss, backward, gradient
all-reduce, Adam step.  K steps are timed between barrier+synchronize fences
and the max over ranks is reported.  ``value`` is whole-job pairs/s.

``--impl reference`` times the reference ALGORITHM in plain PyTorch-ROCm
(4 backbone images per pair, bmm correlation, per-slice conv3d Conv4d), which
is the measured baseline of BASELINE.md (no published numbers exist).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

# RCCL / CUDA-tensor sharing across processes: the ROCm driver only supports
# dmabuf IPC (tests/test_gpu_dist_optim.py, scripts/gpu_job.sh); set before any
# HIP initialisation, inherited by the torchrun children below.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402  (importing torch does not initialise HIP)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Measured reference-algorithm baseline on one MI355X (pairs/s), see BASELINE.md.
BASELINE_PAIRS_PER_S = None
# per-GPU batch of the headline step, sized for the 288 GB HBM of one MI355X
# (BASELINE.json north star and config 3): the throughput-optimal batch of the
# r5 sweep (profiles/r5/batch: 16 -> 764, 128 -> 801, 256 -> 836 pairs/s at
# 57.8 GB, 512 -> 567 at 115 GB); the reference train.py's default batch 16 is
# timed as the train_b16 secondary
HEADLINE_BATCH = 256
# the secondary training records (other sizes / recipes / precisions): train.py's batch
SECONDARY_BATCH = 16
_BASELINE_FILE = os.path.join(ROOT, "profiles", "baseline_reference.json")


def _baseline(batch: int = SECONDARY_BATCH):
    """(reference-algorithm pairs/s per GPU, the per-GPU batch it was measured
    at): the same-batch number when profiles/baseline_reference.json holds one
    ("bf16_pairs_per_s_b<batch>"), else the batch-16 one -- recorded next to
    vs_baseline as baseline_batch, so a cross-batch ratio is never unlabelled."""
    if BASELINE_PAIRS_PER_S is not None:
        return BASELINE_PAIRS_PER_S, SECONDARY_BATCH
    try:
        with open(_BASELINE_FILE) as f:
            rec = json.load(f)
    except Exception:
        return None, None
    key = f"bf16_pairs_per_s_b{batch}"
    if key in rec:
        return float(rec[key]), batch
    return float(rec["pairs_per_s_per_gpu"]), int(rec.get("batch", SECONDARY_BATCH))


def _inloc_secondary():
    """BASELINE configs 3-5 (InLoc dense matching, NC 3,3/16,1, k=2), measured
    after the headline window on rank 0 so the driver's run records them:
    ms/pair at 1600 px and 3200 px in bf16 and in fp16 (IEEE half end to end,
    the reference's half_precision numerics), and 3200 px fp8 (e4m3
    correlation; fused bf16 NC or, in inloc_3200_fp8_nc_fp8, the fp8 Conv4d NC
    kernels)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_inloc
    from ncnet_amd.eval.inloc import INLOC_CUDNN_BENCHMARK
    from ncnet_amd.models import ImMatchNet
    out = {}
    # eval_inloc.py's MIOpen state, not the training headline's solver search
    old_bench = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = INLOC_CUDNN_BENCHMARK
    try:
        torch.manual_seed(0)
        model = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], half_precision=True,
                           relocalization_k_size=2).cuda().eval()
        for name, size, prec in (("inloc_1600_bf16", 1600, "bf16"), ("inloc_3200_bf16", 3200, "bf16"),
                                 ("inloc_1600_fp16", 1600, "fp16"), ("inloc_3200_fp16", 3200, "fp16"),
                                 ("inloc_3200_fp8", 3200, "fp8")):
            # eval_inloc.py's schedule: 10 panos per query, query features extracted once
            r = bench_inloc.run_single(size, pairs=10, warmup=2, model=model, panos_per_query=10, precision=prec)
            r1 = bench_inloc.run_single(size, pairs=3, warmup=1, model=model, panos_per_query=1, precision=prec)
            out[name] = {"ms_per_pair": r["value"], "stages_ms": r["stages_ms"],
                         "stages_ms_eager": r.get("stages_ms_eager"), "panos_per_query": 10,
                         "ms_per_pair_both_backbones": r1["value"], "volume": r["config"]["volume"],
                         "dtype": r["dtype"], "pair_graph": r["pair_graph"]}
            if "pair_graph_error" in r:
                out[name]["pair_graph_error"] = r["pair_graph_error"]
        # the all-fp8 pipeline (fp8 Conv4d NC kernels instead of the fused bf16 stack)
        from ncnet_amd import config as _config
        with _config.override(nc_fp8=True):
            r = bench_inloc.run_single(3200, pairs=10, warmup=2, model=model, panos_per_query=10, precision="fp8")
            out["inloc_3200_fp8_nc_fp8"] = {"ms_per_pair": r["value"], "stages_ms": r["stages_ms"],
                                            "stages_ms_eager": r.get("stages_ms_eager"),
                                            "panos_per_query": 10, "dtype": r["dtype"],
                                            "pair_graph": r["pair_graph"]}
        del model
    except Exception as e:  # the headline record must still print
        out["error"] = repr(e)
    torch.backends.cudnn.benchmark = old_bench
    torch.cuda.empty_cache()
    return out


def train_tflop_per_pair(size: int, ks=(5, 5, 5), ch=(16, 16, 1)) -> float:
    """Useful FLOPs of one training pair at ``size`` px (BASELINE.md's
    accounting): ResNet-101 to layer3 on the 2 images (44.6 GFLOP at 400 px,
    scaling with the pixel count), the positive and rolled-negative
    correlations, and per volume (positive and negative, both symmetric
    branches) every Conv4d forward, data gradient (not for the first layer:
    no gradient flows into the frozen trunk) and weight gradient."""
    n = size // 16
    trunk = 2 * 44.6e9 * (size / 400.0) ** 2
    corr = 2 * 2.0 * n ** 4 * 1024
    fwd, bwd, cin = 0.0, 0.0, 1
    for li, (k, c) in enumerate(zip(ks, ch)):
        f = 2.0 * n ** 4 * cin * c * k ** 4
        fwd += f
        bwd += f * (1 if li == 0 else 2)
        cin = c
    return (trunk + corr + 2 * 2 * (fwd + bwd)) / 1e12


def _train_secondary(batch: int, size: int, ks=(5, 5, 5), ch=(16, 16, 1), steps: int = 5, warmup: int = 2):
    """The headline step (Trainer.train_step, trunk prefetch) at another
    ``--image_size`` or NeighConsensus recipe (the reference trains the IVD /
    InLoc model with --ncons_kernel_sizes 3 3 --ncons_channels 16 1,
    /root/reference/README.md:41-49); reports pairs/s and useful TFLOP/s."""
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.ops import _ext
    from ncnet_amd.parallel.dist import DistContext
    dev = torch.device("cuda")
    torch.manual_seed(4)
    model = ImMatchNet(ncons_kernel_sizes=list(ks), ncons_channels=list(ch), dtype="bf16").to(dev)
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    trainer = Trainer(model, make_adam(params, 5e-4), DistContext(device=dev))
    g = torch.Generator(device=dev).manual_seed(97)
    pool = [{"source_image": torch.randn(batch, 3, size, size, device=dev, generator=g),
             "target_image": torch.randn(batch, 3, size, size, device=dev, generator=g)} for _ in range(2)]
    for w in range(warmup):
        trainer.train_step(pool[w % 2], pool[(w + 1) % 2])
    torch.cuda.synchronize()
    d0 = dict(_ext.DISPATCH)
    t0 = time.perf_counter()
    for i in range(steps):
        loss = trainer.train_step(pool[(warmup + i) % 2], pool[(warmup + i + 1) % 2])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pps = batch * steps / dt
    tf = train_tflop_per_pair(size, ks, ch)
    from ncnet_amd.ops.neigh_consensus import fast1x_ok, layer_kinds
    n = size // 16
    fast = fast1x_ok(layer_kinds(list(ch), list(ks)), list(ch), list(ks),
                     torch.empty(1, 1, n, n, n, n, device=dev), True)
    out = {"pairs_per_s": round(pps, 3), "ms_per_step": round(1e3 * dt / steps, 3), "image_size": size,
           "ncons": [list(ks), list(ch)], "tflop_per_pair": round(tf, 4), "useful_tflops": round(pps * tf, 1),
           "fast_1ch_path": bool(fast), "final_loss": float(loss.detach()),
           "nc_paths": {k: v - d0.get(k, 0) for k, v in _ext.DISPATCH.items() if v != d0.get(k, 0)}}
    del trainer, model
    torch.cuda.empty_cache()
    return out


def _nc_precision_secondary(batch: int, size: int, nc_precision: str, steps: int = 5, warmup: int = 2):
    """The headline step with ``ImMatchNet(nc_precision=...)``: 'fp32' runs every
    NeighConsensus conv, data gradient and weight gradient as a bf16x3 split
    (the reference trains the NC in fp32: /root/reference/lib/conv4d.py:21-24,
    /root/reference/train.py:110-156) -- the mode to use when the weak-loss
    signal is below bf16 resolution (profiles/r2_quality)."""
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import DistContext
    dev = torch.device("cuda")
    torch.manual_seed(3)
    model = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16",
                       nc_precision=nc_precision).to(dev)
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    trainer = Trainer(model, make_adam(params, 5e-4), DistContext(device=dev))
    g = torch.Generator(device=dev).manual_seed(98)
    pool = [{"source_image": torch.randn(batch, 3, size, size, device=dev, generator=g),
             "target_image": torch.randn(batch, 3, size, size, device=dev, generator=g)} for _ in range(2)]
    for w in range(warmup):
        trainer.train_step(pool[w % 2], pool[(w + 1) % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = trainer.train_step(pool[i % 2], pool[(i + 1) % 2])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"pairs_per_s": round(batch * steps / dt, 3), "ms_per_step": round(1e3 * dt / steps, 3),
           "nc_precision": nc_precision, "final_loss": float(loss.detach())}
    del trainer, model
    torch.cuda.empty_cache()
    return out


def _fe_finetune_secondary(batch: int, size: int, steps: int = 5, warmup: int = 2):
    """train.py --fe_finetune_params 1 (last layer3 bottleneck trainable,
    train.py:60-63): the trunk runs under autograd and the L2-norm,
    correlation and MutualMatching backward and the NC input gradient join the
    step; one GPU, same config as the headline."""
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import DistContext
    dev = torch.device("cuda")
    torch.manual_seed(2)
    model = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(dev)
    for p in model.FeatureExtraction.model[-1][-1].parameters():
        p.requires_grad = True
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    trainer = Trainer(model, make_adam(params, 5e-4), DistContext(device=dev))
    g = torch.Generator(device=dev).manual_seed(99)
    pool = [{"source_image": torch.randn(batch, 3, size, size, device=dev, generator=g),
             "target_image": torch.randn(batch, 3, size, size, device=dev, generator=g)} for _ in range(2)]
    for w in range(warmup):
        trainer.train_step(pool[w % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = trainer.train_step(pool[i % 2])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"pairs_per_s": round(batch * steps / dt, 3), "ms_per_step": round(1e3 * dt / steps, 3),
           "trainable_params": sum(p.numel() for p in params), "final_loss": float(loss.detach())}
    del trainer, model
    torch.cuda.empty_cache()
    return out


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(args, argv) -> int:
    """``python bench.py --gpus N`` (N > 1) without a launcher: run the same
    command under ``torch.distributed.run --nproc-per-node N`` as a CHILD
    process (never an exec: this process has not touched the GPU and stays
    that way), relay rank 0's JSON record, and fail loudly when the child fails
    or reports another world size.  Decided from argv/env only, before any
    torch.cuda call."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, NCNET_BENCH_SELF_LAUNCHED="1")
    print(f"bench.py: --gpus {args.gpus} without WORLD_SIZE; launching {' '.join(cmd[1:4])} ...", file=sys.stderr,
          flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    recs = []
    for line in proc.stdout:
        if line.startswith("{") and '"metric"' in line:
            recs.append(line.strip())
        else:
            sys.stdout.write(line)
            sys.stdout.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: torchrun child exited with {rc}", file=sys.stderr)
        return rc if rc > 0 else 1
    if len(recs) != 1:
        print(f"bench.py: expected one JSON record from rank 0, got {len(recs)}", file=sys.stderr)
        return 1
    rec = json.loads(recs[0])
    if rec.get("n_gpus") != args.gpus:
        print(f"bench.py: child reported n_gpus={rec.get('n_gpus')} != --gpus {args.gpus}", file=sys.stderr)
        return 1
    print(recs[0], flush=True)
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=HEADLINE_BATCH,
                    help=f"pairs per GPU (default {HEADLINE_BATCH}: sized for HBM; train.py's default is 16)")
    ap.add_argument("--image-size", type=int, default=400)
    ap.add_argument("--impl", choices=["hip", "reference"], default="hip")
    ap.add_argument("--ref-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--profile", type=str, default="", help="write a torch.profiler trace to this dir")
    ap.add_argument("--only-secondary", type=str, default="",
                    help="debug: skip the headline and print one secondary record "
                         "(nc_fp32 | nc_mixed | fe_finetune | train | train_ivd, at --image-size)")
    ap.add_argument("--lr", type=float, default=5e-4,
                    help="Adam learning rate (train.py's 5e-4).  Diagnostics only: the kernels' clocks depend on the "
                         "data, which drifts with the weights, so same-box kernel A/Bs whose numerics differ in the "
                         "last bits compare at --lr 0 (identical weights every step, the optimizer still runs)")
    ap.add_argument("--inloc", type=int, default=1,
                    help="1: after the timed training steps of a 1-GPU run, also time the InLoc inference configs "
                         "(BASELINE configs 3-5: 1600 px bf16, 3200 px bf16, 3200 px fp8) into config.secondary")
    args = ap.parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(args, argv)
    if args.only_secondary:
        fn = {"nc_fp32": lambda: _nc_precision_secondary(args.batch, args.image_size, "fp32", args.steps, args.warmup),
              "nc_mixed": lambda: _nc_precision_secondary(args.batch, args.image_size, "mixed", args.steps,
                                                          args.warmup),
              "fe_finetune": lambda: _fe_finetune_secondary(args.batch, args.image_size, args.steps, args.warmup),
              "train": lambda: _train_secondary(args.batch, args.image_size, steps=args.steps, warmup=args.warmup),
              "train_ivd": lambda: _train_secondary(args.batch, args.image_size, (3, 3), (16, 1), args.steps,
                                                    args.warmup)}
        print(json.dumps({"secondary": args.only_secondary, **fn[args.only_secondary]()}), flush=True)
        return 0

    from ncnet_amd import config as _config
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import (GradBucket, all_reduce_max_float, barrier, broadcast_module, comm_info,
                                         init_distributed)

    ctx = init_distributed()
    if ctx.world_size != args.gpus:
        # the record must describe the job that ran: never time one rank of a
        # job that was asked for N (or N ranks of a job asked for 1)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ctx.world_size}")
    torch.manual_seed(1)
    torch.backends.cudnn.benchmark = True
    dev = ctx.device
    model = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(dev)
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    broadcast_module(model, ctx)
    # the reference baseline keeps the reference's optimizer (train.py:71:
    # torch.optim.Adam); the HIP path uses FlatAdam (engine/optim.py)
    opt = make_adam(params, args.lr) if args.impl == "hip" else torch.optim.Adam(params, lr=args.lr)

    # a small pool of synthetic batches (random normalised images), generated on device
    gen = torch.Generator(device=dev).manual_seed(1234 + ctx.rank)   # (CPU: gloo smoke runs only)
    s = args.image_size
    pool = [{"source_image": torch.randn(args.batch, 3, s, s, device=dev, generator=gen),
             "target_image": torch.randn(args.batch, 3, s, s, device=dev, generator=gen)} for _ in range(2)]

    if args.impl == "hip":
        trainer = Trainer(model, opt, ctx)

        def step(batch, nxt):
            # exactly train.py's step (Trainer.train_step): the backbone of the
            # next batch is queued on a side stream behind this step (one
            # backbone pass per step), gradient all-reduce, guarded Adam
            return trainer.train_step(batch, nxt)
    else:
        bucket = GradBucket(params, ctx, opt)
        from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_weak_loss
        alg = ReferenceAlgorithm(model, torch.float32 if args.ref_dtype == "fp32" else torch.bfloat16)

        def step(batch, nxt):
            opt.zero_grad(set_to_none=True)
            loss = reference_weak_loss(alg, batch)
            loss.backward()
            if hasattr(opt, "mark_loss"):
                opt.mark_loss(loss)
            bucket.allreduce()
            opt.step()
            return loss

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    npool = len(pool)
    for w in range(args.warmup):
        loss = step(pool[w % npool], pool[(w + 1) % npool])
    sync()
    barrier(ctx)
    sync()

    prof = None
    if args.profile and ctx.is_main:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    # (the pool alternates, so timed step 0 takes the batch the last warmup
    # step prefetched; the window holds exactly K backbone passes)
    for it in range(args.steps):
        j = args.warmup + it
        loss = step(pool[j % npool], pool[(j + 1) % npool])
    sync()
    barrier(ctx)
    sync()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile, exist_ok=True)
        with open(os.path.join(args.profile, "torch_profile.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    elapsed = all_reduce_max_float(elapsed, ctx)

    ms_per_step = 1000.0 * elapsed / args.steps
    pairs_per_s = args.batch * ctx.world_size * args.steps / elapsed
    base, base_batch = _baseline(args.batch)
    # vs_baseline = value / the BASELINE.md number (the reference algorithm
    # measured on ONE MI355X, at this per-GPU batch when measured there, else
    # at batch 16: see baseline_batch); per-GPU ratio = vs_baseline / n_gpus.
    vs = None
    if base:
        vs = pairs_per_s / base
    secondary = None
    # the secondary records are single-GPU measurements: taken in the 1-GPU run
    # only, so the multi-GPU scaling runs stay short and rank 0 never works on
    # alone while its peers tear the process group down
    if args.inloc and ctx.world_size == 1 and dev.type == "cuda" and args.impl == "hip":
        secondary = _inloc_secondary()
        try:
            secondary["fe_finetune_1"] = _fe_finetune_secondary(SECONDARY_BATCH, s)
        except Exception as e:  # the headline record must still print
            secondary["fe_finetune_1"] = {"error": repr(e)}
        try:
            secondary["train_nc_fp32"] = _nc_precision_secondary(SECONDARY_BATCH, s, "fp32")
        except Exception as e:  # the headline record must still print
            secondary["train_nc_fp32"] = {"error": repr(e)}
        try:
            secondary["train_nc_mixed"] = _nc_precision_secondary(SECONDARY_BATCH, s, "mixed")
        except Exception as e:  # the headline record must still print
            secondary["train_nc_mixed"] = {"error": repr(e)}
        # the training step at the other --image_size values and the IVD recipe
        for name, size, ks, ch in (("train_320", 320, (5, 5, 5), (16, 16, 1)),
                                   ("train_480", 480, (5, 5, 5), (16, 16, 1)),
                                   ("train_ivd_400", 400, (3, 3), (16, 1))):
            try:
                secondary[name] = _train_secondary(SECONDARY_BATCH, size, ks, ch)
            except Exception as e:  # the headline record must still print
                secondary[name] = {"error": repr(e)}
        # the headline step at the reference train.py's batch 16 (the headline
        # of rounds 1-4), next to the HBM-sized headline batch
        if args.batch != SECONDARY_BATCH:
            try:
                secondary["train_b16"] = _train_secondary(SECONDARY_BATCH, s, steps=10, warmup=3)
            except Exception as e:  # the headline record must still print
                secondary["train_b16"] = {"error": repr(e)}
        secondary["headline_useful_tflops"] = round(pairs_per_s / ctx.world_size * train_tflop_per_pair(s), 1)
    if ctx.is_main:
        rec = {
            "metric": "image-pairs/sec fwd+bwd, ResNet-101+NC-Net(5,5,5) 400x400 bf16",
            "value": round(pairs_per_s, 3),
            "unit": "image-pairs/s",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if vs is None else round(vs, 3),
            "dtype": "bf16" if args.impl == "hip" or args.ref_dtype == "bf16" else "fp32",
            "data": "synthetic (random normalised 400x400 pairs, random-init weights)",
            "config": {"model": "ResNet-101(layer3)+NC-Net ncons 5,5,5/16,16,1", "global_batch": args.batch * ctx.world_size,
                       "per_gpu_batch": args.batch, "seq_len": None, "image_size": s,
                       "parallelism": f"dp{ctx.world_size}", "impl": args.impl,
                       "baseline_pairs_per_s_1gpu": base, "baseline_batch": base_batch,
                       "final_loss": float(loss.detach()),
                       "comm": comm_info(ctx),
                       "launcher": ("self-launched torchrun" if os.environ.get("NCNET_BENCH_SELF_LAUNCHED")
                                    else "torchrun" if os.environ.get("TORCHELASTIC_RUN_ID") else "python"),
                       "optimizer": type(opt).__name__, "lr": args.lr,
                       "hbm_peak_gb": (round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
                                       if dev.type == "cuda" else None),
                       "runtime": _config.RUNTIME.as_dict(),
                       "secondary": secondary},
        }
        print(json.dumps(rec), flush=True)
    from ncnet_amd.parallel.dist import destroy
    destroy(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
