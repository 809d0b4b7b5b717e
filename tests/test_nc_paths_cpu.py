"""``ops/neigh_consensus.py select_path``: the one place that picks a
NeighConsensus execution path (the table in that module's docstring), checked
on CPU tensors with ``_ext.use_hip`` forced on -- the GPU tests run the paths
themselves.  Reference semantics of every path: lib/model.py:122-153."""
import importlib

import pytest
import torch

from ncnet_amd import config as _config
from ncnet_amd.ops import _ext

nc = importlib.import_module("ncnet_amd.ops.neigh_consensus")


@pytest.fixture
def hip(monkeypatch):
    monkeypatch.setattr(_ext, "use_hip", lambda t: True)
    yield


def _ws(ks, ch, grad=False):
    ws, cin = [], 1
    for k, c in zip(ks, ch):
        ws.append(torch.zeros(k, c, cin, k, k, k, requires_grad=grad))
        cin = c
    return ws


def _x(shape=(1, 1, 6, 6, 6, 6), grad=False):
    return torch.zeros(shape, requires_grad=grad)


def test_cpu_tensors_take_the_reference():
    assert nc.select_path(_x(), _ws((3, 3), (16, 1)), (16, 1)) == "reference"


def test_inference_and_training_paths(hip):
    ivd = ((3, 3), (16, 1))
    pf = ((5, 5, 5), (16, 16, 1))
    with torch.no_grad():
        assert nc.select_path(_x(), _ws(*ivd), ivd[1]) == "fused"
        assert nc.select_path(_x(), _ws(*pf), pf[1]) == "bf16"            # no fused kernel for 5,5,5
        assert nc.select_path(_x(), _ws(*ivd), ivd[1], fp8=True) == "fused"   # fp8 corr + bf16 fused NC
        with _config.override(nc_fp8=True):
            assert nc.select_path(_x(), _ws(*ivd), ivd[1], fp8=True) == "fused_fp8"
            # the fused e4m3 kernel needs the symmetric square volume
            assert nc.select_path(_x((1, 1, 6, 6, 5, 7)), _ws(*ivd), ivd[1], fp8=True) == "fp8"
            assert nc.select_path(_x(), _ws(*ivd), ivd[1], symmetric=False, fp8=True) == "fp8"
            assert nc.select_path(_x(), _ws(*pf), pf[1], fp8=True) == "fp8"
        with _config.override(nc_fused=False):
            assert nc.select_path(_x(), _ws(*ivd), ivd[1]) == "bf16"
        assert nc.select_path(_x(), _ws(*pf), pf[1], precision="fp32") == "x3_inference"
        assert nc.select_path(_x(), _ws(*ivd), ivd[1], precision="mixed") == "x3_inference"
    # training (autograd through the weights)
    assert nc.select_path(_x(), _ws(*ivd, grad=True), ivd[1]) == "bf16"
    assert nc.select_path(_x(), _ws(*pf, grad=True), pf[1], padded=torch.zeros(1)) == "bf16_padded"
    assert nc.select_path(_x(), _ws(*pf, grad=True), pf[1], precision="fp32") == "x3_fused"
    assert nc.select_path(_x(), _ws(*pf, grad=True), pf[1], precision="mixed") == "mixed"
    # mixed off the fused x3 shapes (non-square volume) trains on the full x3 stack
    assert nc.select_path(_x((1, 1, 6, 6, 5, 7)), _ws(*pf, grad=True), pf[1], precision="mixed") == "x3"
    assert nc.select_path(_x(grad=True), _ws(*pf), pf[1], precision="fp32", symmetric=False) == "x3"


def test_unsupported_kernel_size(hip):
    assert nc.select_path(_x(), _ws((4, 4), (16, 1)), (16, 1)) == "torch_fallback"


def test_model_asks_the_same_selector(hip):
    """ImMatchNet.process_correlation takes its fused-inference shortcut exactly
    when select_path answers fused / fused_fp8 (no predicate of its own)."""
    src = importlib.import_module("ncnet_amd.models.immatchnet")
    import inspect
    body = inspect.getsource(src.ImMatchNet.process_correlation)
    assert "select_path" in body and "fused_applies" not in body
