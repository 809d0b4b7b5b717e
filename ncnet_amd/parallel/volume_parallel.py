"""Volume parallelism: one image pair's 4D correlation volume sharded over ranks.

The NC-Net "sequence" is the 4D volume, (hA*wA) x (hB*wB) cells; the
reference only shrinks it on one GPU (relocalization pooling, fp16, batch 1;
SURVEY.md 5.7).  This is the context-parallel analog (SURVEY.md 2.5, 5.7 d):
ranks own contiguous slabs of the (pooled) A-rows ``iA`` and the pipeline
stays exact:

1. features: rank 0 runs the trunk on image A, rank 1 on image B (rank 0 does
   both on one rank), and the L2-normalised packed features are broadcast
   (uint8 view, so bf16 and OCP fp8 operands travel alike);
2. correlation (+ the fused k=2 relocalization pool) of the rank's A-rows
   against all of B: the volume slab is produced in place, never gathered;
3. MutualMatching: the max over B positions of an A cell is local; the max
   over A positions of a B cell is a ``MAX`` all-reduce of a [hB, wB] map;
4. NeighConsensus: the whole Conv4d stack needs sum(k_l // 2) rows of context
   on each side, so ONE halo exchange of the 1-channel input volume with the
   neighbouring ranks (point-to-point, ``batch_isend_irecv`` over RCCL/xGMI)
   is enough: the stack runs on the padded slab and the central rows are
   kept.  At the global volume edges there is no halo and the kernels'
   zero padding is exactly the reference's per-layer padding; at interior
   slab edges the rows polluted by the slab's zero padding are exactly the
   ones cropped.  Symmetric mode works unchanged (the swapped branch convolves
   the slab along its k/l axes and along its i axis with the same padding);
5. MutualMatching again; then the slabs (and relocalization offsets) are
   gathered for match extraction.

Inference only (no autograd through the halo exchange).  Traffic per pair:
features once, two [hB, wB] max-reductions, 2 x sum(k//2) halo rows of the
1-channel volume per neighbour, and the final gather.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import reference as ref
from ..ops.correlation import correlation, correlation_pool2, maxpool4d
from .dist import DistContext


def shard_rows(n_rows: int, world: int, min_rows: int = 1):
    """Balanced contiguous row ranges [(i0, i1)] per rank; ranks beyond the
    point where a slab would be thinner than ``min_rows`` get empty slabs."""
    active = max(1, min(world, n_rows // max(1, min_rows)))
    base, extra = divmod(n_rows, active)
    out, i0 = [], 0
    for r in range(world):
        n = (base + (1 if r < extra else 0)) if r < active else 0
        out.append((i0, i0 + n))
        i0 += n
    return out


def _bcast_bytes(t: torch.Tensor | None, shape, dtype, src: int, ctx: DistContext) -> torch.Tensor:
    if ctx.rank != src:
        t = torch.empty(shape, dtype=dtype, device=ctx.device)
    if ctx.enabled:
        dist.broadcast(t.view(torch.uint8), src)
    return t


def mutual_matching_sharded(c: torch.Tensor, ctx: DistContext) -> torch.Tensor:
    """MutualMatching of an A-row slab [b,1,ni,j,k,l] of the global volume
    (lib/model.py:155-175), with the reference's parenthesisation."""
    b, ch, i, j, k, l = c.shape
    c_b = c.reshape(b, i * j, k, l)
    c_a = c.reshape(b, i, j, k * l)
    if i * j > 0:
        max_over_a = c_b.amax(dim=1, keepdim=True)
    else:
        max_over_a = torch.full((b, 1, k, l), float("-inf"), device=c.device, dtype=c.dtype)
    if ctx.enabled:
        max_over_a = max_over_a.contiguous()
        dist.all_reduce(max_over_a, op=dist.ReduceOp.MAX)
    if i * j == 0:
        return c
    max_over_b = c_a.amax(dim=3, keepdim=True)
    ratio_b = (c_b / (max_over_a + ref.MUTUAL_EPS)).reshape(b, 1, i, j, k, l)
    ratio_a = (c_a / (max_over_b + ref.MUTUAL_EPS)).reshape(b, 1, i, j, k, l)
    return c * (ratio_a * ratio_b)


def exchange_halo(x: torch.Tensor, halo: int, slabs, ctx: DistContext):
    """Pad an A-row slab [b,1,ni,...] with up to ``halo`` rows of each
    neighbouring slab.  Returns (padded, rows added on top)."""
    r = ctx.rank
    i0, i1 = slabs[r]
    if not ctx.enabled or halo == 0 or i1 == i0:
        return x, 0
    prev_ok = r > 0 and slabs[r - 1][1] > slabs[r - 1][0]
    nxt_ok = r + 1 < len(slabs) and slabs[r + 1][1] > slabs[r + 1][0]
    up = min(halo, slabs[r - 1][1] - slabs[r - 1][0]) if prev_ok else 0
    down = min(halo, slabs[r + 1][1] - slabs[r + 1][0]) if nxt_ok else 0
    n_up_send = min(halo, i1 - i0) if prev_ok else 0
    n_down_send = min(halo, i1 - i0) if nxt_ok else 0
    shape = list(x.shape)
    top = bot = None
    ops = []
    if prev_ok:
        shape[2] = up
        top = torch.empty(shape, dtype=x.dtype, device=x.device)
        ops.append(dist.P2POp(dist.isend, x[:, :, :n_up_send].contiguous(), r - 1))
        ops.append(dist.P2POp(dist.irecv, top, r - 1))
    if nxt_ok:
        shape[2] = down
        bot = torch.empty(shape, dtype=x.dtype, device=x.device)
        ops.append(dist.P2POp(dist.isend, x[:, :, x.shape[2] - n_down_send:].contiguous(), r + 1))
        ops.append(dist.P2POp(dist.irecv, bot, r + 1))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    parts = [t for t in (top, x, bot) if t is not None]
    return torch.cat(parts, 2), up


def _gather_rows(x: torch.Tensor, slabs, ctx: DistContext) -> torch.Tensor:
    """All-gather A-row slabs [..., ni, ...] (row dim 2) of different heights."""
    if not ctx.enabled:
        return x
    nmax = max(i1 - i0 for i0, i1 in slabs)
    shape = list(x.shape)
    shape[2] = nmax
    buf = torch.zeros(shape, dtype=x.dtype, device=x.device)
    buf[:, :, : x.shape[2]] = x
    outs = [torch.empty_like(buf) for _ in slabs]
    dist.all_gather(outs, buf)
    return torch.cat([o[:, :, : i1 - i0] for o, (i0, i1) in zip(outs, slabs)], 2)


class VolumeParallelMatcher:
    """Sharded ImMatchNet inference for one pair (batch 1): ``forward``
    returns the full processed volume (and relocalization offsets) on every
    rank, identical to ``model(batch)`` on one device."""

    def __init__(self, model, ctx: DistContext):
        self.model = model
        self.ctx = ctx
        ks = model.NeighConsensus.kernel_sizes
        self.halo = sum(k // 2 for k in ks)

    _DTYPES = (torch.bfloat16, torch.float8_e4m3fn, torch.float32, torch.float16)

    @torch.inference_mode()
    def features(self, src: torch.Tensor, tgt: torch.Tensor):
        """Image A's trunk on rank 0, image B's on rank 1; packed features
        broadcast to every rank (with their grid size and dtype)."""
        ctx, m = self.ctx, self.model
        if not ctx.enabled:
            fa, ga = m.extract(src)
            fb, gb = m.extract(tgt)
            return fa, ga, fb, gb
        src_b = 1 if ctx.world_size > 1 else 0
        out = []
        for img, owner in ((src, 0), (tgt, src_b)):
            meta = torch.zeros(4, dtype=torch.int64, device=ctx.device)
            f = None
            if ctx.rank == owner:
                f, (h, w) = m.extract(img)
                f = f.contiguous()
                meta[:] = torch.tensor([h, w, f.shape[-1], self._DTYPES.index(f.dtype)])
            dist.broadcast(meta, owner)
            h, w, c, code = (int(v) for v in meta.tolist())
            f = _bcast_bytes(f, (1, h * w, c), self._DTYPES[code], owner, ctx)
            out += [f, (h, w)]
        return tuple(out)

    @torch.inference_mode()
    def forward(self, tnf_batch):
        ctx, m = self.ctx, self.model
        src, tgt = tnf_batch["source_image"], tnf_batch["target_image"]
        assert src.shape[0] == 1, "volume parallelism shards ONE pair"
        fa, (ha, wa), fb, (hb, wb) = self.features(src, tgt)
        k = m.relocalization_k_size if m.relocalization_k_size > 1 else 1
        rows = ha // k
        slabs = shard_rows(rows, ctx.world_size, max(1, self.halo))
        i0, i1 = slabs[ctx.rank]
        fa_rows = fa.view(1, ha, wa, -1)[:, i0 * k: i1 * k].reshape(1, (i1 - i0) * k * wa, -1)
        delta = None
        if i1 > i0:
            if k == 2 and ha % 2 == 0 and wa % 2 == 0 and hb % 2 == 0 and wb % 2 == 0:
                corr, delta = correlation_pool2(fa_rows, fb, (i1 - i0) * 2, wa, hb, wb)
            else:
                corr = correlation(fa_rows, fb).view(1, 1, (i1 - i0) * k, wa, hb, wb)
                if k > 1:
                    corr, delta = maxpool4d(corr, k)
        else:
            corr = torch.zeros((1, 1, 0, wa // k, hb // k, wb // k), device=fa.device)
        corr = corr.float()
        corr = mutual_matching_sharded(corr, ctx)
        padded, up = exchange_halo(corr, self.halo, slabs, ctx)
        if i1 > i0:
            nc = m.NeighConsensus
            nc.fp8 = m.corr_dtype == "fp8"
            out = nc(padded)[:, :, up: up + (i1 - i0)].float()
        else:
            out = corr
        out = mutual_matching_sharded(out, ctx)
        full = _gather_rows(out.contiguous(), slabs, ctx)
        if k > 1:
            if delta is None:
                delta = tuple(torch.zeros(out.shape, dtype=torch.uint8, device=out.device) for _ in range(4))
            d = torch.stack([t.to(torch.uint8).reshape(out.shape) for t in delta], 0)   # [4, 1, 1, ni, ...]
            d = _gather_rows(d.view(4, 1, *out.shape[2:]), slabs, ctx).view(4, *full.shape)
            return full, tuple(d[q] for q in range(4))
        return full
