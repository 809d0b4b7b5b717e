"""hipBLASLt 1x1 conv with the trunk's fused epilogue (csrc/gemm_lt.hip):
Y = act(X W^T + bias (+ R)) against a plain PyTorch fp32 reference on the same
bf16 operands, with and without the residual / ReLU, untuned and tuned, and the
trunk plan's per-shape auto choice (models/backbones.py FrozenResNetPlan._c1)."""
import pytest
import torch

from ncnet_amd.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("cin,cout,res,relu", [(256, 64, False, True), (64, 256, True, True), (1024, 256, False, True),
                                              (256, 1024, True, True), (512, 1024, False, False)])
@pytest.mark.parametrize("tune", [0, 1])
def test_gemm_lt_matches_fp32(cin, cout, res, relu, tune):
    torch.manual_seed(cin + cout)
    n, h, w = 3, 17, 23
    cl = torch.channels_last
    x = torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(cout, cin, 1, 1, device=DEV) * cin ** -0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(cout, device=DEV)
    r = torch.randn(n, cout, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl) if res else None
    y = torch.full((n, cout, h, w), float("nan"), device=DEV, dtype=torch.bfloat16).contiguous(memory_format=cl)
    _ext.ext().gemm_lt(x, wt, b, r, y, 1 if relu else 0, tune)
    ref = torch.einsum("nchw,oc->nohw", x.double(), wt[:, :, 0, 0].double()) + b.double().view(1, -1, 1, 1)
    if res:
        ref = ref + r.double()
    if relu:
        ref = ref.relu()
    err = (y.double() - ref).abs().max().item()
    assert err <= 2e-2 * max(1.0, ref.abs().max().item()), err


def test_trunk_plan_auto_equals_native():
    """The auto plan (per-shape native / hipBLASLt) computes the native plan's
    features to bf16 rounding (same operands, different summation order)."""
    from ncnet_amd.models.backbones import FrozenResNetPlan, build_trunk, fold_frozen_bn
    torch.manual_seed(0)
    trunk, _, _ = build_trunk("resnet101")
    trunk = trunk.to(DEV).eval()
    folded = fold_frozen_bn(trunk).to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 200, 200, device=DEV)
    outs = {}
    for mode in ("native", "auto"):
        plan = FrozenResNetPlan(folded, torch.bfloat16)
        plan.use_graphs = False
        plan.conv_mode = mode
        with torch.no_grad():
            for _ in range(2):
                outs[mode] = plan(x).float()
        if mode == "auto":
            assert plan.tuned_choices(), "auto made no per-shape choice"
    a, b = outs["native"], outs["auto"]
    rel = ((a - b).norm() / a.norm()).item()
    assert rel < 2e-2, rel
