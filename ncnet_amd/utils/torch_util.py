"""Batch / tensor utilities (reference lib/torch_util.py, lib/py_util.py).

* ``collate_custom``: dict batches whose tensors are stacked and whose other
  values (e.g. variable-length annotation lists) stay Python lists.
* ``BatchToDevice`` (the reference's ``BatchTensorToVars``): move every tensor
  of a dict batch to a device, non-blocking from pinned memory.
* ``softmax_1d`` (``Softmax1D``), ``expand_dim``, ``create_file_path``.
* ``save_checkpoint`` / ``str_to_bool`` are re-exported from
  ``ncnet_amd.engine.checkpoint``.
"""
from __future__ import annotations

import os
from collections.abc import Mapping

import torch
from torch.utils.data import default_collate

from ..engine.checkpoint import save_checkpoint, str_to_bool  # noqa: F401


def collate_custom(batch):
    if isinstance(batch[0], Mapping):
        return {k: collate_custom([d[k] for d in batch]) for k in batch[0]}
    if torch.is_tensor(batch[0]):
        return default_collate(batch)
    return batch


class BatchToDevice:
    def __init__(self, device="cuda", non_blocking: bool = True):
        self.device = torch.device(device)
        self.non_blocking = non_blocking

    def __call__(self, batch: dict) -> dict:
        return {k: (v.to(self.device, non_blocking=self.non_blocking) if torch.is_tensor(v) else v)
                for k, v in batch.items()}


BatchTensorToVars = BatchToDevice   # reference name


def softmax_1d(x: torch.Tensor, dim: int) -> torch.Tensor:
    """Numerically stable softmax along ``dim`` (not in place, unlike the reference)."""
    x = x - x.max(dim, keepdim=True)[0]
    e = torch.exp(x)
    return e / e.sum(dim, keepdim=True)


Softmax1D = softmax_1d   # reference name


def expand_dim(tensor: torch.Tensor, dim: int, desired_dim_len: int) -> torch.Tensor:
    sz = list(tensor.size())
    sz[dim] = desired_dim_len
    return tensor.expand(tuple(sz))


def create_file_path(filename: str):
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
