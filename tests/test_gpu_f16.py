"""GPU: the IEEE-half (fp16) inference kernels -- the reference's
half_precision numerics (eval_inloc.py:50, lib/model.py:253-267) on the f16
MFMA: L2-norm packing, correlation GEMMs (plain / fused 2x2x2x2 max-pool),
MutualMatching's NC-input writer, the fused InLoc NeighConsensus and the
trunk's NHWC convs, each against an fp32 / fp64 PyTorch reference of the same
op on the same fp16-rounded operands."""
import pytest
import torch
import torch.nn.functional as F

from ncnet_amd.ops import _ext
from ncnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rl2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def test_l2norm_f16():
    from ncnet_amd.ops.correlation import l2norm_pack_f16
    torch.manual_seed(0)
    f = torch.randn(2, 1024, 9, 13, device=DEV)
    y = l2norm_pack_f16(f)
    assert y.dtype == torch.float16 and y.shape == (2, 117, 1024)
    want = ref.feature_l2norm(f).reshape(2, 1024, 117).transpose(1, 2)
    assert rl2(y, want) < 1e-3                     # f16 rounding: 2^-11


@pytest.mark.parametrize("v2", [0, 1])
def test_corr_gemm_f16(v2, tune):
    tune("corr_v2", v2)
    torch.manual_seed(1)
    a = (torch.randn(2, 300, 256, device=DEV) * 0.1).half()
    b = (torch.randn(2, 290, 256, device=DEV) * 0.1).half()
    out = torch.empty(2, 300, 290, device=DEV)
    m = torch.arange(2, device=DEV, dtype=torch.int32)
    _ext.ext().corr_gemm(a, b, out, m, m, 1.0)
    want = torch.bmm(a.double(), b.double().transpose(1, 2))
    assert rl2(out, want) < 1e-5                   # exact products, fp32 sums
    o16 = torch.empty(2, 300, 290, device=DEV, dtype=torch.float16)
    _ext.ext().corr_gemm(a, b, o16, m, m, 1.0)
    assert rl2(o16, want) < 1e-3


def test_corr_pool2_f16_matches_unfused():
    from ncnet_amd.ops.correlation import correlation_pool2
    torch.manual_seed(2)
    fa = torch.nn.functional.normalize(torch.randn(1, 12 * 16, 128, device=DEV), dim=2).half()
    fb = torch.nn.functional.normalize(torch.randn(1, 10 * 14, 128, device=DEV), dim=2).half()
    val, (di, dj, dk, dl) = correlation_pool2(fa, fb, 12, 16, 10, 14)
    full = torch.bmm(fa.float(), fb.float().transpose(1, 2)).view(1, 1, 12, 16, 10, 14)
    want, _ = ref.maxpool4d(full, 2)
    assert rl2(val, want) < 1e-5


def test_mm_nc_input_f16():
    from ncnet_amd.ops.mutual import mutual_matching_nc_input
    torch.manual_seed(3)
    c = torch.rand(2, 1, 7, 9, 7, 9, device=DEV)
    x2 = mutual_matching_nc_input(c, torch.float16)
    assert x2.dtype == torch.float16
    m = ref.mutual_matching(c.double()).reshape(2, 7, 9, 7, 9)
    assert rl2(x2[:2], m) < 1e-3
    assert rl2(x2[2:], m.permute(0, 3, 4, 1, 2)) < 1e-3


def test_fused_nc_f16_vs_fp64():
    from ncnet_amd.ops.neigh_consensus import neigh_consensus_fused_x2
    torch.manual_seed(4)
    V, I, J = 1, 10, 12
    x = torch.rand(V, 1, I, J, I, J, device=DEV)
    w1 = ref.conv4d_weight_from_std(torch.randn(16, 1, 3, 3, 3, 3, device=DEV) * 0.2)
    w2 = ref.conv4d_weight_from_std(torch.randn(1, 16, 3, 3, 3, 3, device=DEV) * 0.05)
    b1, b2 = torch.rand(16, device=DEV) * 0.05, torch.rand(1, device=DEV) * 0.05
    xh = x.half()
    x2 = torch.cat((xh.reshape(V, I, J, I, J), xh.reshape(V, I, J, I, J).permute(0, 3, 4, 1, 2)), 0).contiguous()
    y = neigh_consensus_fused_x2(x2, [w1, w2], [b1, b2])
    want = ref.neigh_consensus(xh.double(), [w1.double(), w2.double()], [b1.double(), b2.double()], True)
    e16 = rl2(y, want)
    xb = x.to(torch.bfloat16)
    x2b = torch.cat((xb.reshape(V, I, J, I, J), xb.reshape(V, I, J, I, J).permute(0, 3, 4, 1, 2)), 0).contiguous()
    eb = rl2(neigh_consensus_fused_x2(x2b, [w1, w2], [b1, b2]),
             ref.neigh_consensus(xb.double(), [w1.double(), w2.double()], [b1.double(), b2.double()], True))
    print("fused NC rel err: f16 %.2e  bf16 %.2e" % (e16, eb))
    assert e16 < 3e-3 and e16 < eb / 4, (e16, eb)


@pytest.mark.parametrize("k,stride,cin,cout,res", [(1, 1, 256, 128, False), (3, 1, 128, 128, True),
                                                    (3, 2, 64, 128, False), (1, 1, 512, 1024, True)])
def test_conv2d_nhwc_f16(k, stride, cin, cout, res):
    torch.manual_seed(5)
    cl = torch.channels_last
    x = torch.randn(2, cin, 20, 24, device=DEV).half().contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).half().contiguous(memory_format=cl)
    b = torch.randn(cout, device=DEV) * 0.1
    pad = k // 2
    ho = (20 + 2 * pad - k) // stride + 1
    wo = (24 + 2 * pad - k) // stride + 1
    r = torch.randn(2, cout, ho, wo, device=DEV).half().contiguous(memory_format=cl) if res else None
    y = torch.empty(2, cout, ho, wo, device=DEV, dtype=torch.float16, memory_format=cl)
    _ext.ext().conv2d_nhwc(x, w, b, r, y, stride, pad, 1)
    want = F.conv2d(x.float(), w.float(), b, stride, pad)
    if res:
        want = want + r.float()
    want = want.relu()
    assert rl2(y, want) < 2e-3


def test_inloc_fp16_model_closer_to_fp32_than_bf16():
    """The half_precision InLoc forward (bf16 trunk; fp16 features, correlation
    + pool, MutualMatching output and fused NC) is closer to the fp32 reference
    algorithm than the bf16 path, with an fp32 trunk under both so the
    comparison isolates the matching stages (the reference halves after its
    fp32 trunk: lib/model.py:263-265)."""
    from ncnet_amd.data.datasets import synthetic_correspondence_batch
    from ncnet_amd.engine.reference_impl import ReferenceAlgorithm, reference_inloc_forward
    from ncnet_amd.models import ImMatchNet
    torch.manual_seed(0)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], relocalization_k_size=2).to(DEV).eval()
    for p in m.NeighConsensus.parameters():
        if p.dim() == 1:
            p.data.uniform_(0.0, 0.1)
    alg = ReferenceAlgorithm(m, torch.float32)
    b = synthetic_correspondence_batch(1, 640, DEV, seed=9)
    with torch.inference_mode():
        r, _ = reference_inloc_forward(alg, b["source_image"], b["target_image"], 2, nc_dtype=torch.float32)
        errs = {}
        for prec in ("bf16", "fp16"):
            m.corr_dtype, m.compute_dtype = prec, torch.float32
            c, _ = m(b)
            errs[prec] = rl2(c, r.float())
    print("InLoc-config volume rel err vs fp32:", errs)
    assert errs["fp16"] < errs["bf16"] / 2, errs
    m.compute_dtype = torch.bfloat16          # the production fp16 mode: still a valid volume
    with torch.inference_mode():
        m.corr_dtype = "fp16"
        c, _ = m(b)
    assert torch.isfinite(c).all() and rl2(c, r.float()) < 3e-2
