"""The reference ALGORITHM in plain PyTorch-ROCm: the measured baseline.

The reference repository publishes no throughput numbers, so
bench.py measures this module on the same MI355X instead.  It reproduces what
lib/model.py + lib/conv4d.py + train.py execute, op for op:

* ``FeatureExtraction`` on the source and the target images, then again on
  the rolled source for the negative pass (4 backbone images per pair,
  train.py:121,137-138);
* ``torch.bmm`` correlation (lib/model.py:110-113);
* torch ``MutualMatching`` (lib/model.py:155-175);
* Conv4d as the per-slice conv3d loop, I*k cuDNN/MIOpen launches per layer
  (lib/conv4d.py:39-48), symmetric branch via permute (lib/model.py:147);
* softmax / max / mean weak loss (train.py:110-156).

``dtype`` selects fp32 (what the reference trains in) or bf16 autocast.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ..ops import reference as ref


class ReferenceAlgorithm(nn.Module):
    def __init__(self, model, dtype: torch.dtype = torch.float32, conv=None):
        """``model`` is an ImMatchNet; its parameters are shared.  ``conv``:
        the Conv4d implementation -- default the reference's per-slice conv3d
        loop (what the baseline times); ``ops.reference.conv4d`` computes the
        same sums with k conv3d calls per layer (numerics checks)."""
        super().__init__()
        self.m = model
        self.dtype = dtype
        self.conv = conv or ref.conv4d_sliced

    def _fe(self, img):
        with torch.autocast("cuda", dtype=self.dtype, enabled=img.is_cuda and self.dtype != torch.float32):
            with torch.no_grad():
                f = self.m.FeatureExtraction.model(img)
        return ref.feature_l2norm(f.float())

    def forward(self, batch):
        fa = self._fe(batch["source_image"])
        fb = self._fe(batch["target_image"])
        with torch.autocast("cuda", dtype=self.dtype, enabled=fa.is_cuda and self.dtype != torch.float32):
            corr = ref.correlation_4d(fa, fb)
            corr = ref.mutual_matching(corr)
            layers = self.m.NeighConsensus.conv_layers()
            ws = [l.weight_ref() for l in layers]
            bs = [l.bias for l in layers]
            corr = ref.neigh_consensus(corr, ws, bs, symmetric=True, conv=self.conv)
            corr = ref.mutual_matching(corr)
        return corr.float()


def reference_weak_loss(alg: ReferenceAlgorithm, batch) -> torch.Tensor:
    """train.py:110-156 including the in-place source roll."""
    b = batch["source_image"].shape[0]
    pos = ref.match_score(alg(batch))
    batch = dict(batch)
    batch["source_image"] = batch["source_image"][np.roll(np.arange(b), -1)]
    neg = ref.match_score(alg(batch))
    return neg - pos


def reference_inloc_forward(alg: ReferenceAlgorithm, src: torch.Tensor, tgt: torch.Tensor, k_size: int = 2,
                            nc_dtype: torch.dtype = torch.float16):
    """eval_inloc.py's forward as the reference executes it: fp32 (or alg.dtype)
    backbone on both images, then ``.half()`` volume (lib/model.py:265-267),
    torch.bmm correlation of the full-resolution volume, the k^4-slice
    maxpool4d (lib/model.py:177-191, batch 1), MutualMatching, the per-slice
    conv3d NeighConsensus and MutualMatching -- the InLoc baseline."""
    fa = alg._fe(src).to(nc_dtype)
    fb = alg._fe(tgt).to(nc_dtype)
    corr = ref.correlation_4d(fa, fb)
    delta = None
    if k_size > 1:
        corr, delta = ref.maxpool4d(corr, k_size)
    corr = ref.mutual_matching(corr)
    layers = alg.m.NeighConsensus.conv_layers()
    ws = [l.weight_ref().to(nc_dtype) for l in layers]
    bs = [l.bias.to(nc_dtype) for l in layers]
    corr = ref.neigh_consensus(corr, ws, bs, symmetric=True, conv=ref.conv4d_sliced)
    corr = ref.mutual_matching(corr)
    return corr, delta
