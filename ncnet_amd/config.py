"""Typed view of the framework's runtime configuration.

The CLIs keep the reference's argparse flags (Appendix A); the execution
toggles are environment variables read HERE, once, when the op modules are
imported (``RUNTIME``) -- the op modules read no environment themselves --
and the dataclass is logged so a run records exactly which code paths it used
(bench.py puts it in its JSON).  The kernel launchers' tuning switches
(non-temporal stores, group-plane tiles per workgroup, A/B kernel variants)
live in csrc/common.h NcnetTuning, seeded from NCNET_* once and changed
in-process with ``_ext.ext().set_tuning``.
"""
from __future__ import annotations

import dataclasses
import os


@dataclasses.dataclass(frozen=True)
class RuntimeConfig:
    nc_encoding: str = "ij"          # 1-channel NC layers: ij encoding (csrc/jshift.hip), the only one
    trunk_plan: bool = True          # NCNET_TRUNK_PLAN
    trunk_graph: bool = True         # NCNET_TRUNK_GRAPH
    force_torch: bool = False        # NCNET_FORCE_TORCH
    allow_torch_fallback: bool = False  # NCNET_ALLOW_TORCH_FALLBACK
    fused_adam: bool = False         # NCNET_FUSED_ADAM
    gp_tpw: int = 5                  # NCNET_GP_TPW: output j-tiles per workgroup of the group-plane conv
    nt_store: bool = True            # NCNET_NT_STORE: non-temporal Conv4d epilogue stores
    bwd_overlap: bool = True         # NCNET_BWD_OVERLAP: NC weight gradients on a side stream
    trunk_prefetch: bool = True      # NCNET_TRUNK_PREFETCH: next batch's frozen backbone on a side stream
    nc_fused: bool = True            # NCNET_NC_FUSED: fused (3,3)/(<=16,1) inference NeighConsensus kernel
    step_priority: bool = False      # NCNET_STEP_PRIORITY: training step on high-priority streams, the
                                     # prefetched trunk at default priority (fills gaps instead of time-slicing)
    prefetch_at: int = 0             # NCNET_PREFETCH_AT: when the next batch's trunk is queued on its stream:
                                     # 0 with the forward, 1 before the backward, 2 after the backward

    @classmethod
    def from_env(cls, env=None) -> "RuntimeConfig":
        e = os.environ if env is None else env
        return cls(trunk_plan=e.get("NCNET_TRUNK_PLAN", "1") != "0",
                   trunk_graph=e.get("NCNET_TRUNK_GRAPH", "1") != "0",
                   force_torch=e.get("NCNET_FORCE_TORCH", "0") == "1",
                   allow_torch_fallback=e.get("NCNET_ALLOW_TORCH_FALLBACK", "0") == "1",
                   fused_adam=e.get("NCNET_FUSED_ADAM", "0") == "1",
                   gp_tpw=int(e.get("NCNET_GP_TPW", "5")),
                   nt_store=e.get("NCNET_NT_STORE", "1") != "0",
                   bwd_overlap=e.get("NCNET_BWD_OVERLAP", "1") == "1",
                   trunk_prefetch=e.get("NCNET_TRUNK_PREFETCH", "1") == "1",
                   nc_fused=e.get("NCNET_NC_FUSED", "1") != "0",
                   step_priority=e.get("NCNET_STEP_PRIORITY", "0") == "1",
                   prefetch_at=int(e.get("NCNET_PREFETCH_AT", "0")))

    def as_dict(self) -> dict:
        return dataclasses.asdict(self)


RUNTIME = RuntimeConfig.from_env()
# one-pass row + column statistics (csrc/volume.hip stats2d) in MutualMatching
# and the weak loss; NCNET_STATS2D=0 restores the separate row / column kernels (A/B)
STATS2D = os.environ.get("NCNET_STATS2D", "1") != "0"
