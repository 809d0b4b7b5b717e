"""Compiler resource guard for the hot gfx950 kernels (CPU: hipcc cross-compiles).

Every kernel instantiation the training step and the InLoc path launch must
compile with no scratch memory and no spilled VGPRs.  Round 2 regressed here
silently (conv16v3 forward / data-gradient picked up scratch from a release
codegen change); spills cost an HBM round trip per access in the innermost
MFMA loops.  Kernels are matched by name prefix + template arguments as
``ncnet_amd.kernel_resources`` reports them.
"""
import shutil

import pytest

from ncnet_amd import kernel_resources as kr

# (kernel name prefix, template-argument string or None for every instantiation)
HOT = [
    ("conv16v4_fwd_kernel", "5, 5, 1, 25, 25"),     # 16->16 forward (training, 400 px)
    ("conv16v4_fwd_kernel", "5, 5, 2, 25, 25"),     # 16->16 data gradient (training, 400 px)
    ("conv16v4_fwd_kernel", None),                  # every compile-time plane: 15 / 20 / 25, k = 3 / 5, x3
    ("wgrad16v4_kernel", "5, 25, 25"),              # 16->16 weight gradient (training)
    ("wgrad16v4_kernel", None),                     # every compile-time plane, k = 3 / 5
    ("wgrad16v3_kernel", None),                     # general-shape 16->16 weight gradient (fallback)
    ("conv16v3_fwd_kernel", None),                  # general-shape 16->16 (k = 3, 5; fwd / dgrad)
    ("conv16v2_fwd_kernel", None),                  # 1-channel layers (group-plane / block modes)
    ("wgrad16v2_kernel", None),
    ("wgrad16p_kernel", None),
    ("conv1x16_kernel", None),                      # 1 -> 16 on padded 1-channel planes (k 5: 20, 25; k 3: 25)
    ("wgrad1x16_kernel", None),                     # 1-channel-operand weight gradients
    ("corr_gemm", None),                            # correlation GEMMs (bf16 v1 / v2, MX-fp8)
    ("nc_fused_k3_kernel", None),                   # fused InLoc NC
    ("conv2d_nhwc", None),                          # native trunk convs (v1, v2, v3 incl. the bf16x3 mode)
    ("l2norm_rows_kernel", None),
    ("mm_apply_kernel", None),
    ("stats_rows_kernel", None),
    ("stats_cols_kernel", None),
]

pytestmark = [
    pytest.mark.skipif(shutil.which(kr.HIPCC) is None and not __import__("os").path.exists(kr.HIPCC),
                       reason="hipcc not available"),
    # device-only compiles of every source; conv4d_fwd.hip alone takes ~11 min on
    # this 8-CPU container (dozens of fully unrolled instantiations)
    pytest.mark.timeout(2400),
]


@pytest.fixture(scope="module")
def records():
    return kr.analyse_all(jobs=4)


def _match(rec, prefix, args):
    name = kr.short(rec.get("name", rec["mangled"]))
    if not name.startswith(prefix):
        return False
    return args is None or name.endswith(f"<{args}>")


@pytest.mark.parametrize("prefix,args", HOT)
def test_hot_kernels_do_not_spill(records, prefix, args):
    hits = [r for r in records if _match(r, prefix, args)]
    assert hits, f"no compiled kernel matches {prefix}<{args}>"
    bad = [(kr.short(r["name"]), r.get("scratch"), r.get("vgpr_spill")) for r in hits
           if r.get("scratch", 0) or r.get("vgpr_spill", 0)]
    assert not bad, f"scratch / VGPR spills in hot kernels: {bad}"


def test_build_remark_cache_is_keyed_on_the_source(tmp_path):
    """kernel_resources reads the release build's remarks only when they were
    produced from the same source, headers and flags (ncnet_amd/build.py
    resource_key); a stale file means a fresh compile."""
    from ncnet_amd import build as b
    src = tmp_path / "zz_cache_probe.hip"
    src.write_text("// probe\n")
    cache = b.resource_cache(src)
    cache.parent.mkdir(exist_ok=True)
    try:
        cache.write_text("# key stale\nremark line\n")
        assert kr._cached_remarks(src) is None
        cache.write_text(f"# key {b.resource_key(src)}\nremark line\n")
        assert kr._cached_remarks(src) == "remark line\n"
        src.write_text("// edited\n")
        assert kr._cached_remarks(src) is None
    finally:
        cache.unlink(missing_ok=True)
