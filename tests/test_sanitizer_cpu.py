"""Sanitizer tier, host side (ncnet_amd/build.py variants).

* every pybind entry point of the extension is called with CPU tensors of
  the right arity and must reject them with a RuntimeError (a TORCH_CHECK in
  bindings.cpp) -- never crash, never reach a launcher;
* the same test, plus the CPU emulation suites, run in a child process on the
  AddressSanitizer build (``_C_asan.so``: bindings and every launcher built
  with ``-fsanitize=address`` by clang) with the clang ASan runtime preloaded:
  a heap/stack error in host code aborts the child with an ASan report.
GPU ASan is not available on this pool; the device side of the sanitizer tier
is the bounds-checked debug build (``NCNET_EXT=debug``, tests/conftest.py).
"""
import importlib
import os
import re
import subprocess
import sys

import pytest
import torch

from ncnet_amd import build as nbuild

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _variant_module():
    variant = os.environ.get("NCNET_EXT", "release")
    name = "ncnet_amd._C" if variant in ("", "release") else f"ncnet_amd._C_{variant}"
    try:
        return importlib.import_module(name)
    except ImportError as e:
        pytest.skip(f"{name} not built ({e})")


def _dummy(kind: str):
    if "Sequence" in kind:
        if "Tensor" in kind:        # tensor lists (reduce_cols): CPU tensors must be rejected too
            return [torch.zeros(16, dtype=torch.float32)]
        return [3, 3, 3] if "SupportsInt" in kind else [0.5, 0.5, 0.5]
    if "Tensor" in kind:
        return None if "None" in kind else torch.zeros(16, dtype=torch.bfloat16)
    if "SupportsFloat" in kind:
        return 1.0
    if "SupportsInt" in kind:
        return 3
    if kind == "bool":
        return True
    raise AssertionError(f"unhandled argument type {kind}")


def test_variant_targets():
    assert nbuild.target_for("release").name == "_C.so"
    assert nbuild.target_for("debug").name == "_C_debug.so"
    assert nbuild.target_for("asan").name == "_C_asan.so"
    with pytest.raises(ValueError):
        nbuild.build(variant="tsan")
    assert os.path.exists(nbuild.asan_runtime())


def test_bindings_reject_cpu_tensors():
    C = _variant_module()
    names = [n for n in dir(C) if not n.startswith("_") and callable(getattr(C, n))]
    assert len(names) >= 20
    for n in names:
        if n in ("set_tuning", "pad_geom"):   # no tensor operands (switches, geometry helper)
            continue
        sig = getattr(C, n).__doc__.strip().splitlines()[0]
        args = re.match(r"\w+\((.*)\) ->", sig).group(1)
        kinds = [a.split(":", 1)[1].split(" = ")[0].strip() for a in re.split(r", (?=\w+:)", args)] if args else []
        with pytest.raises(RuntimeError):
            getattr(C, n)(*[_dummy(k) for k in kinds])


@pytest.mark.slow
def test_cpu_suite_under_asan():
    """The binding test and the CPU kernel-emulation suites on the ASan build."""
    target = nbuild.target_for("asan")
    if not target.exists():
        try:
            nbuild.build(variant="asan")
        except Exception as e:  # pragma: no cover - toolchain missing
            pytest.skip(f"cannot build the ASan variant: {e}")
    env = dict(os.environ)
    pre = env.get("LD_PRELOAD", "")
    env["LD_PRELOAD"] = nbuild.asan_runtime() + (":" + pre if pre else "")
    # python itself is not instrumented: no leak check, no link-order check
    env["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:abort_on_error=1"
    env["NCNET_EXT"] = "asan"
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
           "tests/test_sanitizer_cpu.py::test_bindings_reject_cpu_tensors", "tests/test_kernel_emulation.py",
           "tests/test_nc_general_cpu.py"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "passed" in out
