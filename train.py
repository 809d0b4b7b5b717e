#!/usr/bin/env python
"""Weakly-supervised NC-Net training (reference CLI: train.py:34-47).

Same flags and defaults as the reference, plus:
  --synthetic N        train on N random pairs instead of a CSV dataset
  --num_workers W      data-loader workers per rank (reference: 0 train / 4 test)
  --log_interval L     loss print interval (reference: 1); the values are read
                       back asynchronously (no per-step host sync)
  --sync_log           synchronous per-step loss readback, as the reference
  --resume PATH        real resume: weights + optimizer + epoch + RNG state
  --max_steps S        stop after S training steps (smoke / profiling)
  --metrics PATH       JSONL metrics (rank 0)
  --dtype bf16|fp32    backbone compute dtype of the default (bf16) NC mode
  --nc_precision bf16|mixed|fp32
                       bf16 (default, the headline benchmark): bf16 MFMA operands,
                       fp32 accumulation.  fp32: fp32-accurate training -- fp32
                       trunk, bf16x3 correlation and a bf16x3 NeighConsensus
                       forward AND backward on the fused kernels (~16 mantissa
                       bits per operand).  mixed: the stages the per-stage
                       ablation found necessary (profiles/r5/ablation): the
                       fp32-accurate trunk and NeighConsensus forward, a bf16
                       correlation and bf16 NeighConsensus backward (fp32-class
                       forward numerics at 2/3 of the fp32 mode's NC work).

Which precision to train with: bf16 unless you need fp32-class numerics.  A
per-stage ablation over 24 seeds in the hardest offline regime (random-init
trunk, per-step loss ~1e-8; profiles/r5/ablation/README.md) found the run
either takes off (PCK ~0.7) or its ReLUs die, at rates within noise of each
other for bf16 (10/24), mixed (12/24) and fp32 (13/24): the earlier few-seed
finding that only fp32 learns there did not hold.  mixed / fp32 keep the
reference's fp32 forward numerics (parity studies, checkpoints compared
bit-closely against fp32 training) at 2.2x / 2.9x the bf16 step time.
"""
from __future__ import annotations

import argparse
import datetime
import os
import sys
import time

# RCCL under torchrun: the ROCm driver only supports dmabuf IPC; must be set
# before any HIP initialisation (bench.py does the same).
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import DataLoader, Subset

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ncnet_amd.data import ImagePairDataset, NormalizeImageDict, SyntheticPairDataset  # noqa: E402
from ncnet_amd.data.datasets import collate_uint8_pairs, gpu_pair_batch  # noqa: E402
from ncnet_amd.engine.checkpoint import capture_rng, load_checkpoint, restore_rng, save_checkpoint  # noqa: E402
from ncnet_amd.engine.trainer import AsyncLossLog, Trainer, make_adam  # noqa: E402
from ncnet_amd.models import ImMatchNet  # noqa: E402
from ncnet_amd.parallel.dist import barrier, broadcast_module, destroy, init_distributed, shard_indices  # noqa: E402
from ncnet_amd.utils.timing import SegmentTimer, set_active  # noqa: E402


def build_parser():
    p = argparse.ArgumentParser(description="NC-Net training (MI355X)")
    p.add_argument("--checkpoint", type=str, default="")
    p.add_argument("--image_size", type=int, default=400)
    p.add_argument("--dataset_image_path", type=str, default="datasets/pf-pascal/", help="path to PF Pascal dataset")
    p.add_argument("--dataset_csv_path", type=str, default="datasets/pf-pascal/image_pairs/",
                   help="path to PF Pascal training csv")
    p.add_argument("--num_epochs", type=int, default=5, help="number of training epochs")
    p.add_argument("--batch_size", type=int, default=16, help="training batch size (per GPU)")
    p.add_argument("--lr", type=float, default=0.0005, help="learning rate")
    p.add_argument("--ncons_kernel_sizes", nargs="+", type=int, default=[5, 5, 5], help="kernels sizes in neigh. cons.")
    p.add_argument("--ncons_channels", nargs="+", type=int, default=[16, 16, 1], help="channels in neigh. cons")
    p.add_argument("--result_model_fn", type=str, default="checkpoint_adam", help="trained model filename")
    p.add_argument("--result-model-dir", type=str, default="trained_models", help="path to trained models folder")
    p.add_argument("--fe_finetune_params", type=int, default=0, help="number of layers to finetune")
    # extensions
    p.add_argument("--synthetic", type=int, default=0)
    p.add_argument("--num_workers", type=int, default=-1,
                   help="DataLoader decode workers per rank (-1: min(8, cpus per rank) on GPU, 0 on CPU)")
    p.add_argument("--cpu_resize", action="store_true",
                   help="resize/normalise in the workers (reference behaviour) instead of on the GPU")
    p.add_argument("--log_interval", type=int, default=1)
    p.add_argument("--sync_log", action="store_true",
                   help="read every logged loss back synchronously (the reference's float(loss) per step); "
                        "default: asynchronous pinned-memory readback, printed when ready")
    p.add_argument("--resume", type=str, default="")
    p.add_argument("--max_steps", type=int, default=0)
    p.add_argument("--metrics", type=str, default="")
    p.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--nc_precision", type=str, default="bf16", choices=["bf16", "mixed", "fp32"],
                   help="fp32: fp32-accurate training (fp32 trunk, bf16x3 correlation + NeighConsensus fwd/bwd on "
                        "the fused kernels); mixed: fp32-accurate trunk + NeighConsensus forward, bf16 correlation "
                        "and backward (fp32-class forward numerics at ~1/3 less NC cost than fp32). Over 24 seeds "
                        "bf16, mixed and fp32 took off at the same rate (profiles/r5/ablation): there is no evidence "
                        "that either learns where bf16 does not; pick them for forward numerics, not for learning")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--segment_timing", action="store_true")
    p.add_argument("--profile", type=str, default="")
    return p


class _Shard(torch.utils.data.Sampler):
    """Per-rank, per-epoch reshuffled shard (DistributedSampler semantics)."""

    def __init__(self, n, ctx, shuffle=True, seed=1):
        self.n, self.ctx, self.shuffle, self.seed, self.epoch = n, ctx, shuffle, seed, 0

    def set_epoch(self, e):
        self.epoch = e

    def __iter__(self):
        return iter(shard_indices(self.n, self.ctx, self.epoch, self.shuffle, self.seed, drop_last=self.ctx.world_size > 1))

    def __len__(self):
        return self.n // self.ctx.world_size if self.ctx.world_size > 1 else self.n


def main(argv=None):
    args = build_parser().parse_args(argv)
    ctx = init_distributed()
    torch.manual_seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(args.seed)
    np.random.seed(args.seed)
    if ctx.is_main:
        print("ImMatchNet training script (ncnet_amd)")
        print(args)

    # --resume rebuilds the NC architecture from the checkpoint's args, like --checkpoint
    model = ImMatchNet(use_cuda=ctx.device.type == "cuda", checkpoint=(args.resume or args.checkpoint) or None,
                       ncons_kernel_sizes=args.ncons_kernel_sizes, ncons_channels=args.ncons_channels,
                       dtype=args.dtype, nc_precision=args.nc_precision).to(ctx.device)
    # the saved Namespace must describe the architecture actually built
    args.ncons_kernel_sizes = list(model.NeighConsensus.kernel_sizes)
    args.ncons_channels = list(model.NeighConsensus.channels)
    if args.fe_finetune_params > 0:  # train.py:60-63
        for i in range(args.fe_finetune_params):
            for p in model.FeatureExtraction.model[-1][-(i + 1)].parameters():
                p.requires_grad = True
    broadcast_module(model, ctx)
    params = [p for p in model.parameters() if p.requires_grad]
    if ctx.is_main:
        print("Trainable parameters:")
        for i, p in enumerate(params):
            print(f"{i + 1}: {tuple(p.shape)}")
    optimizer = make_adam(params, args.lr)

    size = (args.image_size, args.image_size)
    gpu_resize = ctx.device.type == "cuda" and not args.cpu_resize
    if args.synthetic:
        train_set = SyntheticPairDataset(args.synthetic, size, seed=1)
        test_set = SyntheticPairDataset(max(2 * args.batch_size, args.synthetic // 8), size, seed=2)
    else:
        norm = NormalizeImageDict(["source_image", "target_image"])
        train_set = ImagePairDataset(args.dataset_csv_path, "train_pairs.csv", args.dataset_image_path,
                                     output_size=size, transform=norm, gpu_resize=gpu_resize)
        test_set = ImagePairDataset(args.dataset_csv_path, "val_pairs.csv", args.dataset_image_path,
                                    output_size=size, transform=norm, gpu_resize=gpu_resize)
    tr_sampler = _Shard(len(train_set), ctx, True, args.seed)
    te_sampler = _Shard(len(test_set), ctx, True, args.seed + 7)
    pin = ctx.device.type == "cuda"
    nw = args.num_workers
    if nw < 0:
        nw = min(8, max(1, (os.cpu_count() or 2) // max(1, ctx.world_size) - 1)) if pin else 0
    lkw = dict(batch_size=args.batch_size, num_workers=nw, pin_memory=pin, drop_last=True,
               collate_fn=collate_uint8_pairs if (gpu_resize and not args.synthetic) else None,
               persistent_workers=nw > 0, prefetch_factor=4 if nw > 0 else None)
    train_loader = DataLoader(train_set, sampler=tr_sampler, **lkw)
    test_loader = DataLoader(test_set, sampler=te_sampler, **lkw)
    if gpu_resize and not args.synthetic:
        trainer_to_device = lambda batch: gpu_pair_batch(batch, ctx.device, size[0], size[1])  # noqa: E731
    else:
        trainer_to_device = None

    checkpoint_name = os.path.join(args.result_model_dir,
                                   datetime.datetime.now().strftime("%Y-%m-%d_%H:%M") + "_" + args.result_model_fn +
                                   ".pth.tar")
    train_loss = np.zeros(args.num_epochs)
    test_loss = np.zeros(args.num_epochs)
    best_test_loss = float("inf")
    start_epoch = 1
    if args.resume:
        ck = load_checkpoint(args.resume)
        optimizer.load_state_dict(ck["optimizer"])
        start_epoch = int(ck["epoch"]) + 1
        best_test_loss = float(ck.get("best_test_loss", best_test_loss))
        n = min(len(train_loss), len(ck["train_loss"]))
        train_loss[:n] = ck["train_loss"][:n]
        test_loss[:n] = ck["test_loss"][:n]
        restore_rng(ck.get("rng"))
        checkpoint_name = args.resume
        if ctx.is_main:
            print(f"Resumed from {args.resume} at epoch {start_epoch}")
    if ctx.is_main:
        print("Checkpoint name: " + checkpoint_name)

    timer = SegmentTimer(device=ctx.device) if args.segment_timing else None
    set_active(timer)
    trainer = Trainer(model, optimizer, ctx, metrics_path=args.metrics or None)
    trainer.batch_to_device = trainer_to_device
    if args.max_steps:
        # bounded run (smoke / profiling)
        model.train()
        prof = None
        if args.profile and ctx.is_main:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if ctx.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            prof = torch.profiler.profile(activities=acts)
            prof.__enter__()
        t0 = time.perf_counter()
        t_warm, warm = None, min(10, max(0, args.max_steps - 1))
        steps = 0

        def batches():
            while True:
                for b in train_loader:
                    yield b
        it = batches()
        steplog = AsyncLossLog(ctx.device, sync=args.sync_log)

        def show(recs):
            for r in recs:
                msg = f"step {r['step']} loss {r['loss']:.6f}"
                if "segments_ms" in r:
                    msg += " " + " ".join(f"{k}={v:.2f}ms" for k, v in r["segments_ms"].items())
                print(msg, flush=True)
        nxt = trainer.to_device(next(it))
        while steps < args.max_steps:
            batch = nxt
            # one batch of lookahead, as Trainer.process_epoch: its backbone overlaps this step
            nxt = trainer.to_device(next(it)) if steps + 1 < args.max_steps else None
            loss = trainer.train_step(batch, nxt)
            steps += 1
            if steps == warm:
                if ctx.device.type == "cuda":
                    torch.cuda.synchronize()
                t_warm = time.perf_counter()
            if ctx.is_main and (steps % max(1, args.log_interval) == 0):
                meta = {"step": steps}
                if timer is not None:
                    meta["segments_ms"] = timer.collect()
                show(steplog.push(loss, meta))
            elif ctx.is_main:
                show(steplog.poll())
        if ctx.is_main:
            show(steplog.drain())
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        if prof is not None:
            prof.__exit__(None, None, None)
            os.makedirs(args.profile, exist_ok=True)
            sort = "cuda_time_total" if ctx.device.type == "cuda" else "cpu_time_total"
            with open(os.path.join(args.profile, "train_profile.txt"), "w") as f:
                f.write(prof.key_averages().table(sort_by=sort, row_limit=60))
            prof.export_chrome_trace(os.path.join(args.profile, "train_trace.json"))
        if ctx.is_main:
            t1 = time.perf_counter()
            dt = t1 - t0
            msg = f"{steps} steps in {dt:.2f}s ({steps * args.batch_size * ctx.world_size / dt:.1f} pairs/s)"
            if t_warm is not None and steps > warm:
                # steady state: excludes DataLoader worker start-up and the first (graph-capturing) steps
                msg += (f"; steady state after {warm} steps: "
                        f"{(steps - warm) * args.batch_size * ctx.world_size / (t1 - t_warm):.1f} pairs/s")
            print(msg)
        set_active(None)
        destroy(ctx)
        return

    if ctx.is_main:
        print("Starting training...")
    for epoch in range(start_epoch, args.num_epochs + 1):
        tr_sampler.set_epoch(epoch)
        train_loss[epoch - 1] = trainer.process_epoch("train", epoch, train_loader, args.log_interval, args.sync_log)
        test_loss[epoch - 1] = trainer.process_epoch("test", epoch, test_loader, args.log_interval, args.sync_log)
        is_best = test_loss[epoch - 1] < best_test_loss
        best_test_loss = min(test_loss[epoch - 1], best_test_loss)
        if ctx.is_main:
            save_checkpoint({"epoch": epoch, "args": args, "state_dict": model.state_dict(),
                             "best_test_loss": best_test_loss, "optimizer": optimizer.state_dict(),
                             "train_loss": train_loss, "test_loss": test_loss, "rng": capture_rng()},
                            is_best, checkpoint_name)
        barrier(ctx)
    if ctx.is_main:
        print("Done!")
    set_active(None)
    destroy(ctx)


if __name__ == "__main__":
    main()
