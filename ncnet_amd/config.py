"""Typed runtime configuration of the framework.

The CLIs keep the reference's argparse flags (Appendix A).  Every execution
switch -- which code path runs, and the kernel launchers' tuning table
(csrc/common.h ``NcnetTuning``) -- is a field of ``RuntimeConfig``:

* the ``NCNET_*`` environment variables are read HERE, once, when the package
  is imported (``RUNTIME = RuntimeConfig.from_env()``); no other module reads
  the environment (launcher variables -- RANK, WORLD_SIZE, MASTER_* -- and the
  build script's ROCM_PATH aside);
* the op modules read ``config.RUNTIME.<field>`` at call time, so
  ``with config.override(nc_fp8=True): ...`` switches a path in-process (the
  bench's secondaries, tests);
* the launcher tuning fields are pushed into the extension when it loads and
  on every ``override`` (ops/_ext.py ``apply_tuning``): the C++ side reads no
  environment either;
* ``bench.py`` records ``RUNTIME.as_dict()`` in its JSON, so a record names
  every switch of the code path that produced it.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os


@dataclasses.dataclass(frozen=True)
class RuntimeConfig:
    # -- code paths -----------------------------------------------------------
    trunk_plan: bool = True          # NCNET_TRUNK_PLAN: pre-cast frozen-trunk execution plan (else autocast)
    trunk_graph: bool = True         # NCNET_TRUNK_GRAPH: the trunk plan replayed as one HIP graph
    trunk_conv: str = "auto"         # NCNET_TRUNK_CONV: auto | native | blas (models/backbones.py)
    trunk_fp32: str = "auto"         # NCNET_TRUNK_FP32: the fp32 frozen trunk -- x3 (bf16x3 splits on the
                                     #   native MFMA convs, ~2^-16 relative) | miopen (true fp32) | auto:
                                     #   x3 for nc_precision 'fp32' / 'mixed' training, miopen for corr_dtype='fp32'
                                     #   inference (the reference's evaluation numerics)
    force_torch: bool = False        # NCNET_FORCE_TORCH (with allow_torch_fallback): PyTorch reference ops
    allow_torch_fallback: bool = False  # NCNET_ALLOW_TORCH_FALLBACK: configs without a HIP kernel may run PyTorch
    ext_variant: str = "release"     # NCNET_EXT: release | debug (bounds-checked) | asan build of the extension
    adam: str = "flat"               # NCNET_ADAM: flat (engine/optim.py FlatAdam) | torch | fused
    trunk_prefetch: bool = True      # NCNET_TRUNK_PREFETCH: next batch's frozen backbone on a side stream
    bwd_overlap: bool = True         # NCNET_BWD_OVERLAP: NC weight gradients on a side stream
    nc_fused: bool = True            # NCNET_NC_FUSED: fused (3,3)/(<=16,1) inference NeighConsensus kernel
    cout1_taps: bool = True          # NCNET_COUT1_TAPS: tap-row Cout=1 forward (csrc/cout1.hip) at 25x25 planes, k 5
    nc_fp8: bool = False             # NCNET_NC_FP8: e4m3 NC in fp8 mode: the fused fp8 kernel for the
                                     #   (3,3)/(<=16,1) stack, the fp8 Conv4d kernels for other stacks
    stats2d: bool = True             # NCNET_STATS2D: one-pass row + column statistics (csrc/volume.hip)
    pair_graph: bool = True          # NCNET_PAIR_GRAPH: InLoc pair matching replayed as a HIP graph
    fault_step: int = -1             # NCNET_FAULT_STEP: inject a failure at this training step (tests)
    pg_timeout_s: int = 600          # NCNET_PG_TIMEOUT_S: process-group timeout (rank-failure detector)
    force_pg: bool = False           # NCNET_FORCE_PG: create a process group at world size 1
    dist_backend: str = ""           # NCNET_DIST_BACKEND: override nccl / gloo (rehearsals)
    # -- kernel launcher tuning (csrc/common.h NcnetTuning, A/B only) ---------
    nt_store: int = 1                # NCNET_NT_STORE: non-temporal Conv4d epilogue stores
    gp_tpw: int = 5                  # NCNET_GP_TPW: output j-tiles per group-plane workgroup
    conv_v3: int = 0                 # NCNET_CONV_V3: conv16v3 instead of conv16v4 at the compile-time planes
    wgrad_v3: int = 0                # NCNET_WGRAD_V3: wgrad16v3 instead of wgrad16v4
    wgrad_flags: int = 0             # NCNET_WGRAD_FLAGS: wgrad16v3 ablation flags
    conv2d_variant: int = 0          # NCNET_CONV2D_VARIANT: 0 auto, 1 register-staged, 2 DMA ring
    conv2d_v3: int = 1               # NCNET_CONV2D_V3: chip-round v3 trunk tiles where the auto rule picks them
    corr_v2: int = -1                # NCNET_CORR_V2: -1 auto, 0 / 1 force the correlation GEMM variant
    corr_ns: int = 3                 # NCNET_CORR_NS: ring stages (3 or 4) of corr_gemm_v2
    c1x_pd: int = 2                  # NCNET_C1X_PD: conv1x16 transposed-read lookahead (tiles), 1, 2 or 3
    conv2d_256: int = 1              # NCNET_CONV2D_256: 256 x 256 trunk conv tiles for Cout = 256 (big grids)
    s2d_rt: int = 2                  # NCNET_S2D_RT: stats2d 64-row sub-tiles per block, volumes >= 1024 rows (1/2/4)

    # the launcher tuning fields, in the order of csrc/common.h tuning_slot()
    TUNING = ("nt_store", "gp_tpw", "conv_v3", "wgrad_v3", "wgrad_flags", "conv2d_variant", "conv2d_v3",
              "corr_v2", "corr_ns", "c1x_pd", "conv2d_256", "s2d_rt")

    @classmethod
    def from_env(cls, env=None) -> "RuntimeConfig":
        e = os.environ if env is None else env
        kw = {}
        for f in dataclasses.fields(cls):
            v = e.get("NCNET_" + f.name.upper())
            if v is None:
                continue
            if f.type in ("bool", bool):
                kw[f.name] = v not in ("0", "", "false", "False")
            elif f.type in ("int", int):
                kw[f.name] = int(v)
            else:
                kw[f.name] = v
        return cls(**kw)

    def as_dict(self) -> dict:
        return dataclasses.asdict(self)

    def tuning(self) -> dict:
        return {k: int(getattr(self, k)) for k in self.TUNING}


RUNTIME = RuntimeConfig.from_env()


def set_runtime(cfg: RuntimeConfig) -> None:
    """Replace the process-wide configuration (and push its launcher tuning
    into the extension if it is loaded)."""
    global RUNTIME
    RUNTIME = cfg
    from .ops import _ext
    _ext.apply_tuning()


@contextlib.contextmanager
def override(**fields):
    """``with override(nc_fp8=True): ...`` -- the configuration with these
    fields replaced, restored on exit."""
    old = RUNTIME
    set_runtime(dataclasses.replace(old, **fields))
    try:
        yield RUNTIME
    finally:
        set_runtime(old)
