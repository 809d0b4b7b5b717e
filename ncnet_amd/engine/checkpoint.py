"""Checkpoint I/O in the reference's ``.pth.tar`` layout (train.py:197-205,
lib/torch_util.py:48-61), plus real resume.

Written dict: ``{'epoch', 'args' (argparse.Namespace), 'state_dict',
'best_test_loss', 'optimizer', 'train_loss' (np.ndarray), 'test_loss'
(np.ndarray)}``; resume-only extras (``'rng'``, ``'step'``) are added under
their own keys and ignored by reference tools.

Loading never unpickles arbitrary objects: ``torch.load(weights_only=True)``
with ``argparse.Namespace`` and numpy array reconstruction allow-listed, which
is what reference checkpoints contain (their ``args`` is a pickled
Namespace -- the reason the reference's own loader fails on torch >= 2.6).
"""
from __future__ import annotations

import argparse
import os
import shutil
from os.path import basename, dirname, exists, join

import numpy as np
import torch


def _safe_globals():
    g = [argparse.Namespace, np.ndarray, np.dtype]
    try:
        from numpy._core.multiarray import _reconstruct  # numpy >= 2
    except Exception:  # pragma: no cover
        from numpy.core.multiarray import _reconstruct
    g.append(_reconstruct)
    try:
        import numpy.dtypes as nd

        g += [getattr(nd, n) for n in dir(nd) if n.endswith("DType")]
    except Exception:  # pragma: no cover
        pass
    try:
        from numpy.core.multiarray import scalar  # legacy path name in old pickles
        g.append(scalar)
    except Exception:
        pass
    try:
        from numpy._core.multiarray import scalar as scalar2
        g.append(scalar2)
    except Exception:
        pass
    return g


def load_checkpoint(path: str, map_location="cpu") -> dict:
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def save_checkpoint(state: dict, is_best: bool, file: str, save_all_epochs: bool = False) -> str:
    """Same file naming as lib/torch_util.py:48-61: ``file`` (or
    ``<epoch>_<name>``) and a ``best_<name>`` copy when ``is_best``."""
    model_dir, model_fn = dirname(file), basename(file)
    if model_dir and not exists(model_dir):
        os.makedirs(model_dir, exist_ok=True)
    target = join(model_dir, f"{state['epoch']}_{model_fn}") if save_all_epochs else file
    tmp = target + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, target)
    if is_best:
        shutil.copyfile(target, join(model_dir, "best_" + model_fn))
    return target


def str_to_bool(v: str) -> bool:
    """CLI boolean parser (lib/torch_util.py:64-70), raising the argparse error
    the reference intended."""
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


def capture_rng() -> dict:
    st = {"torch": torch.get_rng_state(), "numpy": np.random.get_state()[1].copy()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def restore_rng(st: dict):
    if not st:
        return
    if "torch" in st:
        torch.set_rng_state(st["torch"])
    if "numpy" in st:
        s = np.random.get_state()
        np.random.set_state((s[0], np.asarray(st["numpy"], dtype=np.uint32), 624, 0, 0.0))
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
