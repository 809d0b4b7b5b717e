"""Weakly-supervised training loop (train.py:110-205), DP-aware.

Differences from the reference, all semantics-preserving:
* the negative pass reuses the positive-pass backbone features rolled by one
  (exact: the backbone is in eval mode and per-sample);
* the loss is read back to the host asynchronously (``AsyncLossLog``: pinned
  copies behind events, printed once complete; no per-step host sync), every
  ``log_interval`` steps; ``sync_log`` restores the reference's synchronous
  per-step ``float(loss)`` (train.py:175-180);
* evaluation (``mode='test'``) runs under ``torch.inference_mode`` (the
  reference builds graphs it never uses, train.py:170-174);
* gradients are averaged over ranks with one bucketed RCCL all-reduce;
* NaN/Inf guard: a step whose loss or gradients are non-finite on any rank
  is skipped exactly (parameters, Adam moments and step untouched), on the
  device for FlatAdam (engine/optim.py);
* with a ``utils.timing.SegmentTimer`` installed (train.py --segment_timing)
  every logged record carries mean per-segment GPU milliseconds.
"""
from __future__ import annotations

import json
import math
import time

import numpy as np
import torch

from .. import config as _config

from ..ops.loss import weak_loss_from_corr
from ..parallel.dist import DistContext, GradBucket, all_reduce_mean
from ..utils.timing import active as active_timer, segment


class AsyncLossLog:
    """Loss readback without host syncs.  ``push`` queues a device scalar:
    a non-blocking copy into pinned host memory and an event behind it on the
    current stream; ``poll`` returns the records whose events have completed
    (``Event.query``, never a wait), in push order, each with the GPU time since
    the log was created (``elapsed_s``, from timing events, so it does not
    drift with the host running ahead).  ``drain`` waits for the rest (epoch
    end).  Without CUDA, or with ``sync=True`` (the reference's synchronous
    ``float(loss)`` per logged step), ``push`` reads the value immediately."""

    def __init__(self, device, sync: bool = False):
        self.cuda = torch.device(device).type == "cuda" and torch.cuda.is_available()
        self.sync = sync or not self.cuda
        self.pending = []
        self.t0 = time.perf_counter()
        self.ev0 = None
        if self.cuda:
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev0.record()

    def push(self, value: torch.Tensor, meta: dict) -> list:
        if self.sync:
            rec = dict(meta, loss=float(value))
            if self.cuda:
                torch.cuda.synchronize()
            rec["elapsed_s"] = time.perf_counter() - self.t0
            return [rec]
        host = torch.empty((), dtype=torch.float32, pin_memory=True)
        host.copy_(value.detach().float().reshape(()), non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.pending.append((host, ev, meta))
        return self.poll()

    def poll(self, block: bool = False) -> list:
        out = []
        while self.pending and (block or self.pending[0][1].query()):
            host, ev, meta = self.pending.pop(0)
            ev.synchronize()
            out.append(dict(meta, loss=float(host), elapsed_s=self.ev0.elapsed_time(ev) / 1e3))
        return out

    def drain(self) -> list:
        return self.poll(block=True)


def make_adam(params, lr: float) -> torch.optim.Optimizer:
    """Adam as in train.py:71.

    Default: ``FlatAdam`` (engine/optim.py) -- flat parameter/gradient
    buffers, the gradient buffer doubles as the RCCL bucket, three HIP
    launches per step and an exact asynchronous NaN/Inf step skip.
    config.RUNTIME.adam (NCNET_ADAM) = 'torch' selects torch.optim.Adam
    (foreach), 'fused' its fused kernel.  The state_dict layout is
    torch.optim.Adam's in every case, so checkpoints interchange."""
    from .optim import FlatAdam

    params = list(params)
    kind = _config.RUNTIME.adam
    if kind == "flat" and params and all(p.dtype == torch.float32 for p in params) \
            and len({p.device for p in params}) == 1:
        return FlatAdam(params, lr=lr)
    fused = kind == "fused" and bool(params) and params[0].is_cuda
    return torch.optim.Adam(params, lr=lr, fused=True) if fused else torch.optim.Adam(params, lr=lr)


def weak_loss(model, batch, normalization: str | None = "softmax", alpha: float = 30) -> torch.Tensor:
    """score_neg - score_pos (train.py:110-156). ``alpha`` is unused, as in the reference."""
    src, tgt = batch["source_image"], batch["target_image"]
    vols = model.weak_loss_volumes(src, tgt)
    return weak_loss_from_corr(vols, src.shape[0], normalization)


def weak_loss_from_features(model, feats, normalization: str | None = "softmax") -> torch.Tensor:
    """weak_loss on backbone features ``(f, (h, w), b)`` from TrunkPrefetcher.take."""
    f, hw, b = feats
    return weak_loss_from_corr(model.weak_loss_volumes_from_features(f, hw, b), b, normalization)


class TrunkPrefetcher:
    """Software pipeline over training steps: the frozen backbone (+ L2-norm
    packing) of batch t+1 runs on a side HIP stream while step t's
    correlation / NeighConsensus forward+backward and optimizer step run on
    the main stream.  The trunk's implicit-GEMM convs leave most of the chip
    idle at 25x25 (layer3), so they fill in behind the NC kernels.

    Every step still runs exactly one backbone pass (for the batch after it),
    so a timed window of K steps contains K backbone passes.  Only valid when
    no backbone parameter is trainable (the reference default,
    ``--fe_finetune_params 0``): the features of batch t+1 must not depend on
    step t's update.  Disabled otherwise, on CPU, and with
    config.RUNTIME.trunk_prefetch off (NCNET_TRUNK_PREFETCH=0); then ``take``
    just runs the backbone in place.
    """

    def __init__(self, model):
        self.model = model
        dev = next(model.parameters()).device
        fe_trainable = any(p.requires_grad for p in model.FeatureExtraction.parameters())
        self.enabled = dev.type == "cuda" and not fe_trainable and _config.RUNTIME.trunk_prefetch
        self.stream = torch.cuda.Stream(device=dev) if self.enabled else None
        self._pending = None

    def _extract(self, batch):
        src, tgt = batch["source_image"], batch["target_image"]
        with torch.no_grad():
            f, hw = self.model.extract(torch.cat((src, tgt), 0))
        return f, hw, src.shape[0]

    def submit(self, batch) -> None:
        """Queue the backbone of ``batch`` (the NEXT step's) on the side stream."""
        self._pending = None
        if not self.enabled or batch is None:
            return
        main = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(main)           # inputs ready; earlier work only
        with torch.cuda.stream(self.stream):
            f, hw, b = self._extract(batch)
            done = torch.cuda.Event()
            done.record(self.stream)
        for t in (batch["source_image"], batch["target_image"]):
            t.record_stream(self.stream)
        self._pending = (batch, f, hw, b, done)

    def take(self, batch):
        """Backbone features of ``batch``: the prefetched ones if ``batch`` is
        the one last submitted, else computed now on the current stream."""
        pend, self._pending = self._pending, None
        if pend is not None and pend[0] is batch:
            _, f, hw, b, done = pend
            main = torch.cuda.current_stream(self.stream.device)
            main.wait_event(done)
            for t in (f if isinstance(f, tuple) else (f,)):    # split (hi, lo) operands in fp32 mode
                t.record_stream(main)
            return f, hw, b
        if self.enabled:                        # batch may have been moved on the prefetch stream
            main = torch.cuda.current_stream(self.stream.device)
            main.wait_stream(self.stream)
            for t in (batch["source_image"], batch["target_image"]):
                t.record_stream(main)
        with segment("backbone"):
            return self._extract(batch)


class Trainer:
    def __init__(self, model, optimizer, ctx: DistContext, normalization="softmax", nan_guard=True,
                 metrics_path: str | None = None, fault_step: int | None = None):
        self.model = model
        self.opt = optimizer
        self.ctx = ctx
        self.normalization = normalization
        self.nan_guard = nan_guard
        params = [p for p in model.parameters() if p.requires_grad]
        # with a trainable backbone (--fe_finetune_params) the NC gradients are
        # all-reduced while autograd is still in the backbone (GradBucket early segment)
        nc = getattr(model, "NeighConsensus", None)
        early = [p for p in nc.parameters() if p.requires_grad] if nc is not None else None
        self.bucket = GradBucket(params, ctx, optimizer, early=early)
        self.flat = getattr(optimizer, "flat_grad", None) is not None
        if self.flat:
            optimizer.guard = nan_guard   # nan_guard=False: FlatAdam applies every step unguarded
        self.metrics_path = metrics_path if ctx.is_main else None
        self.global_step = 0
        self.fault_step = fault_step if fault_step is not None else _config.RUNTIME.fault_step
        self.prefetch = TrunkPrefetcher(model)
        self.batch_to_device = None       # optional hook: host batch -> device batch (train.py: GPU resize)

    def _move(self, batch):
        if self.batch_to_device is not None:
            return self.batch_to_device(batch)
        dev = self.ctx.device
        return {k: (v.to(dev, non_blocking=True) if torch.is_tensor(v) else v) for k, v in batch.items()}

    def to_device(self, batch):
        """Host batch -> device.  With the trunk prefetcher the copies (and a
        ``batch_to_device`` hook such as train.py's GPU resize + normalise) are
        queued on the prefetch stream, in front of that batch's backbone, so they
        overlap the current step instead of delaying it on the main stream."""
        st = self.prefetch.stream if self.prefetch.enabled else None
        if st is None:
            return self._move(batch)
        with torch.cuda.stream(st):
            return self._move(batch)

    def train_step(self, batch, next_batch=None) -> torch.Tensor:
        """One step on ``batch``; ``next_batch`` (already on the device) gets
        its backbone pass queued with this step's forward (TrunkPrefetcher: it
        fills the CUs the forward's kernels leave idle; queued later it only
        competes with the backward's two streams, measured in round 4)."""
        if self.fault_step >= 0 and self.global_step == self.fault_step:
            raise RuntimeError(f"injected fault at step {self.global_step} (NCNET_FAULT_STEP)")
        self.opt.zero_grad(set_to_none=True)
        self.bucket.reset()
        with segment("forward"):
            feats = self.prefetch.take(batch)
            self.prefetch.submit(next_batch)
            loss = weak_loss_from_features(self.model, feats, self.normalization)
        with segment("backward"):
            loss.backward()
        if self.flat and self.nan_guard:
            # loss-finite indicator rides in the gradient bucket: every rank's
            # FlatAdam then skips the same (globally non-finite) step, with no host sync
            self.opt.mark_loss(loss)
        with segment("allreduce"):
            self.bucket.allreduce()
        with segment("optimizer"):
            if self.nan_guard and not self.flat and not self._all_finite(loss):
                self.opt.zero_grad(set_to_none=True)      # skip: params and optimizer state untouched
            else:
                self.opt.step()
        self.global_step += 1
        return loss.detach()

    def _all_finite(self, loss) -> bool:
        """Global finite check for optimizers without the flat guard (host sync)."""
        ok = torch.isfinite(loss.detach()).all()
        for p in self.bucket.params:
            if p.grad is not None:
                ok = ok & torch.isfinite(p.grad).all()
        flag = ok.float().reshape(1)
        if self.ctx.enabled:
            import torch.distributed as dist
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item() > 0)

    @torch.inference_mode()
    def eval_step(self, batch) -> torch.Tensor:
        if self.prefetch.enabled:               # the batch was moved on the prefetch stream
            main = torch.cuda.current_stream(self.prefetch.stream.device)
            main.wait_stream(self.prefetch.stream)
            # the batch was allocated on the prefetch stream but is read here on
            # main: without this, once the caller drops it, the allocator could
            # hand its blocks to the next to_device on the prefetch stream while
            # this step's kernels are still queued (train() does the same in
            # TrunkPrefetcher.take)
            for v in batch.values():
                if torch.is_tensor(v) and v.is_cuda:
                    v.record_stream(main)
        return weak_loss(self.model, batch, self.normalization).detach()

    def _log(self, rec: dict):
        if self.metrics_path:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def process_epoch(self, mode: str, epoch: int, loader, log_interval: int = 1, sync_log: bool = False) -> float:
        """Returns the epoch's mean loss (averaged over ranks).  Every
        ``log_interval``-th step's loss is printed and logged as in the
        reference (train.py:175-180), read back through ``AsyncLossLog`` (no
        per-step host sync; ``sync_log=True``: synchronous, as the reference)."""
        is_train = mode == "train"
        self.model.train(is_train)
        total = torch.zeros((), device=self.ctx.device)
        n = 0
        nb = len(loader)
        it = iter(loader)
        nxt = next(it, None)
        nxt = self.to_device(nxt) if nxt is not None else None
        batch_idx = -1
        log = AsyncLossLog(self.ctx.device, sync=sync_log)

        def emit(recs):
            for rec in recs:
                if self.ctx.is_main:
                    bi = rec["step"]
                    print(f"{mode.capitalize()} Epoch: {epoch} [{bi}/{nb} ({100.0 * bi / max(nb, 1):.0f}%)]"
                          f"\t\tLoss: {rec['loss']:.6f}", flush=True)
                rec["pairs_per_s"] = rec["pairs"] / max(rec["elapsed_s"], 1e-9)
                self._log(rec)

        while nxt is not None:
            batch_idx += 1
            batch = nxt
            nxt = next(it, None)          # one batch of lookahead: its backbone overlaps this step
            nxt = self.to_device(nxt) if nxt is not None else None
            loss = self.train_step(batch, nxt) if is_train else self.eval_step(batch)
            total += loss.float()
            n += 1
            if log_interval and batch_idx % log_interval == 0:
                pairs = n * batch["source_image"].shape[0] * self.ctx.world_size
                meta = {"mode": mode, "epoch": epoch, "step": batch_idx, "pairs": pairs}
                if self.ctx.device.type == "cuda":
                    meta["hbm_peak_gb"] = torch.cuda.max_memory_allocated(self.ctx.device) / 2 ** 30
                timer = active_timer()
                if timer is not None and timer.enabled:
                    meta["segments_ms"] = timer.collect()
                emit(log.push(all_reduce_mean(loss, self.ctx), meta))
            else:
                emit(log.poll())
        emit(log.drain())
        mean = float(all_reduce_mean(total / max(n, 1), self.ctx))
        if self.ctx.is_main:
            print(f"{mode.capitalize()} set: Average loss: {mean:.4f}", flush=True)
        return mean
