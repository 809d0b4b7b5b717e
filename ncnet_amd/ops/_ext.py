"""Loader for the in-tree HIP extension (``ncnet_amd/_C.so``).

Dispatch policy (used by every op in ``ncnet_amd.ops``):

* GPU tensors run the hand-written gfx950 kernels.  If the extension cannot be
  imported on a machine with a GPU the op raises -- there is no silent eager
  fallback (``NCNET_ALLOW_TORCH_FALLBACK=1`` / config.RUNTIME.allow_torch_fallback opts into the PyTorch
  oracle path explicitly, e.g. for A/B debugging).
* CPU tensors run the pure-PyTorch oracles in ``ncnet_amd.ops.reference``.
"""
from __future__ import annotations

import collections

import torch

from .. import config as _config

_C = None
_ERR: Exception | None = None


def load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    try:
        import importlib

        variant = _config.RUNTIME.ext_variant   # build variants: ncnet_amd/build.py
        name = "ncnet_amd._C" if variant in ("", "release") else f"ncnet_amd._C_{variant}"
        _C = importlib.import_module(name)
    except Exception as e:  # pragma: no cover - depends on the build state
        _ERR = e
    apply_tuning()
    return _C


def apply_tuning() -> None:
    """Push config.RUNTIME's launcher tuning fields into the extension's
    process-wide table (csrc/common.h NcnetTuning; the C++ side reads no
    environment)."""
    m = _C
    if m is None or not hasattr(m, "set_tuning"):
        return
    for k, v in _config.RUNTIME.tuning().items():
        m.set_tuning(k, int(v))


def available() -> bool:
    return load() is not None


def fallback_allowed() -> bool:
    return _config.RUNTIME.allow_torch_fallback


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` must go through the HIP kernels."""
    if not t.is_cuda:
        return False
    if fallback_allowed() and _config.RUNTIME.force_torch:
        return False
    if load() is None:
        if fallback_allowed():
            return False
        raise RuntimeError(
            "ncnet_amd HIP extension (_C.so) is not built/importable on a GPU machine; "
            f"run `python -m ncnet_amd.build` (import error: {_ERR!r})")
    return True


def ext():
    m = load()
    if m is None:
        raise RuntimeError(f"ncnet_amd HIP extension unavailable: {_ERR!r}")
    return m


# Which implementation each NC-Net op dispatched to, per process (tests and
# bench.py read it: a GPU run must show HIP paths, never "torch_fallback").
DISPATCH: collections.Counter = collections.Counter()


def count(path: str) -> None:
    DISPATCH[path] += 1


def torch_fallback(what: str) -> None:
    """Called before a GPU op would run a PyTorch oracle instead of a HIP
    kernel: raises unless NCNET_ALLOW_TORCH_FALLBACK=1 (no silent fallbacks)."""
    if not fallback_allowed():
        raise NotImplementedError(
            f"{what}: no HIP kernel for this configuration on the GPU; set NCNET_ALLOW_TORCH_FALLBACK=1 "
            "to run the PyTorch reference path instead")
    count("torch_fallback")
