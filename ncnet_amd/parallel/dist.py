"""Data parallelism over RCCL (``torch.distributed`` backend "nccl" on ROCm).

One process per GPU (torchrun-style env: RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT).  The reference has no distributed code at all
(SURVEY.md section 2.5); this is the new DP-1 component:

* every rank trains on its own shard of pairs, with its own negative roll;
* trainable parameters are broadcast from rank 0 at start;
* after backward, ALL trainable gradients are flattened into one persistent
  fp32 bucket and averaged with a single all-reduce.  The NC-Net gradient is
  720 KB (PF config) -- latency-bound on xGMI, so one bucket issued once is
  the right shape; with ``--fe_finetune_params`` the bucket grows by ~4.5 MB
  per un-frozen bottleneck, still one collective;
* scalar metrics are averaged with a tiny all-reduce only when logged.

On CPU (tests) the same code runs over the gloo backend.
"""
from __future__ import annotations

import datetime
import os
import weakref
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        """True whenever a process group exists -- including world size 1
        under torchrun, so the RCCL collectives really execute there too."""
        return dist.is_available() and dist.is_initialized()


def wants_process_group(world: int) -> bool:
    """A process group is created for WORLD_SIZE > 1, for any torchrun launch
    (TORCHELASTIC_RUN_ID is set by torch.distributed.run, also at
    --nproc-per-node 1) and when NCNET_FORCE_PG=1.  A plain ``python bench.py``
    stays collective-free."""
    if world > 1:
        return True
    from .. import config as _config
    if _config.RUNTIME.force_pg:
        return True
    return bool(os.environ.get("TORCHELASTIC_RUN_ID"))


def init_distributed(device: str | None = None, timeout_s: int | None = None) -> DistContext:
    """Initialise from the environment (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_*).  Without a launcher (``wants_process_group`` False) this is a
    single-process context with no process group.

    ``timeout_s`` (default config.RUNTIME.pg_timeout_s: NCNET_PG_TIMEOUT_S or 600) is the rank-failure
    detector: a collective that a dead or hung rank never joins raises on the
    surviving ranks after that many seconds instead of hanging forever."""
    from .. import config as _config
    if timeout_s is None:
        timeout_s = _config.RUNTIME.pg_timeout_s
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = (device != "cpu") and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    backend = "none"
    if wants_process_group(world):
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = "nccl" if use_gpu else "gloo"
        # config.RUNTIME.dist_backend (NCNET_DIST_BACKEND=gloo): rehearse the multi-rank
        # GPU path with several ranks on ONE card (RCCL refuses two ranks per device)
        backend = _config.RUNTIME.dist_backend or backend
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if use_gpu and backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        backend = dist.get_backend()
    return DistContext(rank, world, local, dev, backend)


def comm_info(ctx: DistContext) -> dict:
    """What actually carried the collectives (recorded in bench/metrics JSON)."""
    info = {"backend": dist.get_backend() if ctx.enabled else "none", "world_size": ctx.world_size,
            "process_group": bool(ctx.enabled)}
    if ctx.enabled and info["backend"] == "nccl":
        try:
            v = torch.cuda.nccl.version()
            info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception:  # pragma: no cover
            info["rccl_version"] = None
    return info


def broadcast_parameters(params, ctx: DistContext, src: int = 0):
    """Broadcast tensors (parameters, or a module's whole state) from ``src``.

    Pass ``model.state_dict().values()`` (or use ``broadcast_module``) so the
    frozen backbone and BN statistics are identical on every rank too."""
    if not ctx.enabled:
        return
    with torch.no_grad():
        for p in params:
            dist.broadcast(p.data if hasattr(p, "data") else p, src)


def broadcast_module(module: torch.nn.Module, ctx: DistContext, src: int = 0):
    broadcast_parameters(list(module.state_dict().values()), ctx, src)


class GradBucket:
    """One flat fp32 gradient bucket for a fixed list of parameters.

    With a ``FlatAdam`` optimizer (engine/optim.py) the bucket IS the
    optimizer's flat gradient buffer (the ``.grad`` tensors are views into
    it): the all-reduce runs in place, with no pack/unpack copies, and the
    1/world average is folded into the Adam kernel (``grad_scale``).  The
    buffer's trailing slot carries the loss-finite indicator, so the NaN guard
    sees every rank's loss.  Other optimizers get a private bucket with
    pack -> all-reduce -> average -> unpack.
    """

    def __init__(self, params, ctx: DistContext, optimizer=None, early=None):
        self.params = [p for p in params if p.requires_grad]
        self.ctx = ctx
        self.inplace = getattr(optimizer, "flat_grad", None) is not None
        self._work = None
        self._hooks = []            # post-accumulate hook handles of the early segment
        self._armed = False
        self._early = []            # in-flight early segment all-reduces
        self._early_seg = None      # (lo, hi) flat range reduced early, or None
        if self.inplace:
            self.flat = optimizer.flat_grad
            optimizer.grad_scale = 1.0 / ctx.world_size if ctx.enabled else 1.0
            if early and ctx.enabled:
                self._arm_early(optimizer, [p for p in early if p.requires_grad])
            return
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)

    def _arm_early(self, optimizer, early):
        """Overlap: ``early`` parameters (the NeighConsensus weights, whose
        gradients are final as soon as the NC backward ends) are all-reduced
        from a post-accumulate hook while autograd continues into the backbone
        (``--fe_finetune_params``); ``finish`` then reduces the rest.  Their
        span of the flat buffer must be contiguous and must not hold the
        loss-indicator slot (FlatAdam lays parameters out in order, the slot last)."""
        spans = {id(p): sp for p, sp in zip(optimizer.params, optimizer.spans)}
        if not early or len(early) == len(self.params) or any(id(p) not in spans for p in early):
            return
        lo = min(spans[id(p)][0] for p in early)
        hi = max(spans[id(p)][0] + spans[id(p)][1] for p in early)
        if hi - lo != sum(p.numel() for p in early):
            return                                    # not contiguous: plain single bucket
        self._early_seg = (lo, hi)
        self._pending = set()
        ids = {id(p) for p in early}
        me = weakref.ref(self)      # the parameters must not keep a dropped bucket alive

        def hook(p):
            b = me()
            if b is None or not b._armed or id(p) not in ids or b._early_seg is None:
                return
            b._pending.discard(id(p))
            if not b._pending and not b._early:
                b._early.append(dist.all_reduce(b.flat[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
                b.early_launches += 1

        self._ids = ids
        self.early_launches = 0
        self._hooks = [p.register_post_accumulate_grad_hook(hook) for p in early]
        self.reset()

    def reset(self):
        """Arm the early segment for the next backward (Trainer: before backward).
        Hooks fire only between ``reset`` and ``finish``: a backward that this
        bucket does not own launches nothing."""
        if self._early_seg is not None:
            self._pending = set(self._ids)
            self._early = []
            self._armed = True

    def close(self):
        """Remove the early-segment hooks (a replacement bucket on the same
        parameters must not find this one's hooks still firing)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self._armed = False

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover  (interpreter teardown)
            pass

    def start(self):
        """Launch the (async) all-reduce (packing the grads first unless in place)."""
        if not self.ctx.enabled:
            return
        if self._early_seg is not None:
            lo, hi = self._early_seg
            if not self._early:                       # hooks did not fire (no grads flowed): reduce it now
                self._early.append(dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
            # the rest: [0, lo) and [hi, end) (the latter holds the loss slot)
            rest = [self.flat[:lo]] if lo > 0 else []
            rest.append(self.flat[hi:])
            self._work = [dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True) for t in rest]
            return
        if not self.inplace:
            off = 0
            for p in self.params:
                n = p.numel()
                if p.grad is None:
                    self.flat[off:off + n].zero_()
                else:
                    self.flat[off:off + n].copy_(p.grad.reshape(-1))
                off += n
        self._work = dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, async_op=True)

    def finish(self):
        """Wait (and, for a private bucket, scatter the averaged gradients back)."""
        self._armed = False
        if not self.ctx.enabled or self._work is None:
            return
        for w in (self._work if isinstance(self._work, list) else [self._work]) + self._early:
            w.wait()
        self._work = None
        self._early = []
        if self.inplace:
            return
        self.flat.div_(self.ctx.world_size)
        off = 0
        for p in self.params:
            n = p.numel()
            g = self.flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone().to(p.dtype)
            else:
                p.grad.copy_(g)
            off += n

    def allreduce(self):
        self.start()
        self.finish()


def all_reduce_mean(value: torch.Tensor, ctx: DistContext) -> torch.Tensor:
    if not ctx.enabled:
        return value
    v = value.detach().clone().float()
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    return v / ctx.world_size


def all_reduce_max_float(x: float, ctx: DistContext) -> float:
    if not ctx.enabled:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(ctx: DistContext):
    if ctx.enabled:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def shard_indices(n: int, ctx: DistContext, epoch: int = 0, shuffle: bool = True, seed: int = 1,
                  drop_last: bool = True) -> list[int]:
    """DistributedSampler-style disjoint per-rank shard of range(n)."""
    if shuffle:
        g = torch.Generator().manual_seed(seed + epoch)
        order = torch.randperm(n, generator=g).tolist()
    else:
        order = list(range(n))
    per = n // ctx.world_size if drop_last else -(-n // ctx.world_size)
    if not drop_last:
        order = order + order[: per * ctx.world_size - n]
    return order[ctx.rank * per:(ctx.rank + 1) * per]


def destroy(ctx: DistContext):
    if ctx.enabled:
        dist.destroy_process_group()
