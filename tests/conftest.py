import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def set_runtime(monkeypatch, **fields):
    """Switch ncnet_amd.config.RUNTIME fields for one test (the op modules read
    the configuration at call time; launcher tuning goes to the extension)."""
    import dataclasses
    from ncnet_amd import config
    monkeypatch.setattr(config, "RUNTIME", dataclasses.replace(config.RUNTIME, **fields))
    from ncnet_amd.ops import _ext
    _ext.apply_tuning()


@pytest.fixture
def runtime(monkeypatch):
    """``runtime(nc_fp8=True)`` inside a test: see set_runtime."""
    yield lambda **kw: set_runtime(monkeypatch, **kw)
    from ncnet_amd.ops import _ext
    monkeypatch.undo()
    _ext.apply_tuning()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _ncnet_debug_kernel_checks(request):
    """With NCNET_EXT=debug (the bounds-checked kernel build, ncnet_amd/build.py
    --debug) a GPU test fails if any kernel printed an NCNET_CHECK line."""
    if os.environ.get("NCNET_EXT") != "debug" or "gpu" not in request.keywords or not torch.cuda.is_available():
        yield
        return
    capfd = request.getfixturevalue("capfd")
    yield
    torch.cuda.synchronize()
    out, err = capfd.readouterr()
    sys.stdout.write(out)
    sys.stderr.write(err)
    if "NCNET_CHECK failed" in out + err and "selftest" not in request.node.name:
        pytest.fail("device bounds check failed:\n" + "\n".join(
            ln for ln in (out + err).splitlines() if "NCNET_CHECK" in ln)[:4000])


@pytest.fixture
def tune(monkeypatch):
    """tune(name, value): set a launcher tuning field of config.RUNTIME (pushed
    into csrc/common.h NcnetTuning by the set_tuning binding) for this test;
    restored afterwards."""
    from ncnet_amd.ops import _ext
    yield lambda name, value: set_runtime(monkeypatch, **{name: int(value)})
    monkeypatch.undo()
    _ext.apply_tuning()
