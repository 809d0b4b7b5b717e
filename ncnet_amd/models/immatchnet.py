"""ImMatchNet (NC-Net) with the reference's constructor and forward API.

Reference: lib/model.py:19-282.  Module names (``FeatureExtraction.model``,
``NeighConsensus.conv.{0,2,4}``) and parameter shapes match the reference so
``.pth.tar`` checkpoints load unchanged.

Compute policy (MI355X):
* the frozen backbone runs in eval mode under ``no_grad``, bf16, channels-last
  (MIOpen); frozen BN is optionally folded into the convs;
* L2-norm + operand packing, correlation GEMM, MutualMatching, the Conv4d
  stack and the loss reductions run on the hand-written HIP kernels;
* ``half_precision`` (the reference's InLoc setting) runs the correlation and
  the NeighConsensus on IEEE-half operands (f16 MFMA, fp32 accumulation);
  otherwise the NC path runs bf16 operands, or, by ``nc_precision``, the
  fp32-accurate bf16x3 split ('fp32') or its fp32-forward / bf16-backward mix
  ('mixed'), and ``corr_dtype='fp8'`` selects the e4m3 inference path.
"""
from __future__ import annotations

import importlib
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import reference as ref
from ..ops.conv4d import Conv4d
from ..ops.correlation import (correlation, correlation_pool2, correlation_x3, l2norm_pack, l2norm_pack_f16,
                               l2norm_pack_fp8, l2norm_pack_split, maxpool4d as _maxpool4d)
from ..ops import _ext as _ext_mod
from ..ops.mutual import (mutual_matching, mutual_matching_nc_input as _mm_nc_input,
                          mutual_matching_padded as _mm_padded)
from ..ops.neigh_consensus import neigh_consensus

# the module (the package re-exports the function under the same name)
_nc_ops = importlib.import_module("ncnet_amd.ops.neigh_consensus")
_ext_count = _ext_mod.count
from ..utils.timing import segment
from .backbones import FrozenResNetPlan, FrozenResNetPlanX3, build_trunk, fold_frozen_bn, load_trunk_state

from .. import config as _config


def _ext_available() -> bool:
    from ..ops import _ext
    return _ext.available()


def featureL2Norm(feature: torch.Tensor) -> torch.Tensor:  # noqa: N802 (reference name)
    return ref.feature_l2norm(feature)


def MutualMatching(corr4d: torch.Tensor) -> torch.Tensor:  # noqa: N802 (reference name)
    return mutual_matching(corr4d)


def maxpool4d(corr4d_hres: torch.Tensor, k_size: int = 4):
    """Returns (corr4d, max_i, max_j, max_k, max_l) like lib/model.py:177-191,
    but batch-correct and with integer offsets."""
    vals, (di, dj, dk, dl) = _maxpool4d(corr4d_hres, k_size)
    return vals, di, dj, dk, dl


class FeatureExtraction(nn.Module):
    def __init__(self, train_fe: bool = False, feature_extraction_cnn: str = "resnet101",
                 feature_extraction_model_file: str = "", normalization: bool = True, last_layer: str = "",
                 use_cuda: bool = True):
        super().__init__()
        self.normalization = normalization
        self.feature_extraction_cnn = feature_extraction_cnn
        self.model, self.out_channels, self.stride = build_trunk(feature_extraction_cnn, last_layer)
        if feature_extraction_model_file:
            sd = torch.load(feature_extraction_model_file, map_location="cpu", weights_only=True)
            load_trunk_state(self.model, sd, feature_extraction_cnn)
        if not train_fe:
            for p in self.model.parameters():
                p.requires_grad = False
        if use_cuda and torch.cuda.is_available():
            self.model = self.model.cuda()
        self._folded = None
        self._folded_version = None
        # the fp32 frozen trunk: 'x3' (bf16x3 plan, ~2^-16 relative, the fp32-accurate
        # training mode) or 'miopen' (true fp32, the reference's evaluation numerics);
        # ImMatchNet sets it from nc_precision / corr_dtype, config.RUNTIME.trunk_fp32 overrides
        self.fp32_trunk = "miopen"

    def trunk_forward(self, images: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
        """Raw (un-normalised) trunk features, channels-last on GPU."""
        frozen = not any(p.requires_grad for p in self.model.parameters())
        x = images
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        if frozen and not self.training and x.is_cuda and self.feature_extraction_cnn.startswith("resnet"):
            rt = _config.RUNTIME
            if dtype in (torch.bfloat16, torch.float16) and rt.trunk_plan:
                return self._plan(dtype)(x)
            x3 = rt.trunk_fp32 == "x3" or (rt.trunk_fp32 == "auto" and self.fp32_trunk == "x3")
            if dtype == torch.float32 and rt.trunk_plan and x3 and _ext_available():
                # fp32-accurate trunk as bf16x3 splits on the native MFMA convs
                return self._plan(torch.float32)(x)
            net = self._folded_trunk()
        else:
            net = self.model
        use_amp = x.is_cuda and dtype in (torch.bfloat16, torch.float16)
        with torch.autocast("cuda", dtype=dtype, enabled=use_amp):
            with torch.set_grad_enabled(torch.is_grad_enabled() and not frozen):
                return net(x)

    def _folded_trunk(self):
        ver = sum(p._version for p in self.model.parameters()) + sum(b._version for b in self.model.buffers())
        if self._folded is None or self._folded_version != ver:
            self._folded = fold_frozen_bn(self.model).to(memory_format=torch.channels_last)
            self._folded_version = ver
        return self._folded

    def _plan(self, dtype):
        ver = sum(p._version for p in self.model.parameters()) + sum(b._version for b in self.model.buffers())
        key = (ver, dtype)
        if getattr(self, "_plan_key", None) != key:
            if dtype == torch.float32:
                self._plan_obj = FrozenResNetPlanX3(self._folded_trunk())
            else:
                self._plan_obj = FrozenResNetPlan(self._folded_trunk(), dtype)
            self._plan_key = key
        return self._plan_obj

    def forward(self, image_batch: torch.Tensor) -> torch.Tensor:
        features = self.trunk_forward(image_batch)
        if self.normalization:
            features = featureL2Norm(features.float())
        return features


class FeatureCorrelation(nn.Module):
    """'4D' (used by ImMatchNet) and legacy '3D' correlation (lib/model.py:89-120)."""

    def __init__(self, shape: str = "3D", normalization: bool = True):
        super().__init__()
        self.normalization = normalization
        self.shape = shape
        self.ReLU = nn.ReLU()

    def forward(self, feature_A, feature_B):  # noqa: N803
        if self.shape == "3D":
            corr = ref.correlation_3d(feature_A, feature_B)
        else:
            b, c, ha, wa = feature_A.shape
            _, _, hb, wb = feature_B.shape
            fa = feature_A.permute(0, 2, 3, 1).reshape(b, ha * wa, c)
            fb = feature_B.permute(0, 2, 3, 1).reshape(b, hb * wb, c)
            corr = correlation(fa, fb).view(b, 1, ha, wa, hb, wb)
        if self.normalization:
            corr = featureL2Norm(self.ReLU(corr))
        return corr


class NeighConsensus(nn.Module):
    def __init__(self, use_cuda: bool = True, kernel_sizes=(3, 3, 3), channels=(10, 10, 1),
                 symmetric_mode: bool = True):
        super().__init__()
        self.symmetric_mode = symmetric_mode
        self.kernel_sizes = list(kernel_sizes)
        self.channels = list(channels)
        mods = []
        for i, (k, c) in enumerate(zip(kernel_sizes, channels)):
            cin = 1 if i == 0 else channels[i - 1]
            mods.append(Conv4d(in_channels=cin, out_channels=c, kernel_size=k, bias=True))
            mods.append(nn.ReLU(inplace=True))
        self.conv = nn.Sequential(*mods)
        if use_cuda and torch.cuda.is_available():
            self.conv.cuda()

    def conv_layers(self):
        return [m for m in self.conv if isinstance(m, Conv4d)]

    def forward(self, x, padded=None):
        """``padded``: x's zero-padded bf16 planes of both symmetric branches
        (ops/mutual.py mutual_matching_padded), used by the bf16 training stack."""
        layers = self.conv_layers()
        ws = [m.weight_ref() for m in layers]
        bs = [m.bias if m.bias is not None else torch.zeros(m.out_channels, device=x.device) for m in layers]
        return neigh_consensus(x, ws, bs, self.channels, symmetric=self.symmetric_mode,
                               fp8=getattr(self, "fp8", False), precision=getattr(self, "precision", "bf16"),
                               padded=padded)

    def padded_input_ks(self, x) -> int:
        """Kernel size of the first layer when the bf16 training stack will take
        its padded-plane path on ``x`` (MutualMatching then writes the planes
        directly), else 0."""
        if not (self.symmetric_mode and x.is_cuda and getattr(self, "precision", "bf16") == "bf16"
                and not getattr(self, "fp8", False) and torch.is_grad_enabled()):
            return 0
        kinds = _nc_ops.layer_kinds(self.channels, self.kernel_sizes)
        if kinds is None or not _nc_ops.fast1x_ok(kinds, self.channels, self.kernel_sizes, x, True):
            return 0
        return self.kernel_sizes[0]


def _load_reference_checkpoint(path: str):
    from ..engine.checkpoint import load_checkpoint

    ck = load_checkpoint(path)
    ck["state_dict"] = OrderedDict((k.replace("vgg", "model"), v) for k, v in ck["state_dict"].items())
    return ck


_MAPS: dict = {}


def _pair_maps(b: int, device):
    """Batch index maps of the positive pairs (a_i, b_i) followed by the rolled
    negatives (a_{i+1}, b_i) (train.py:137), cached per (b, device)."""
    key = (b, str(device))
    m = _MAPS.get(key)
    if m is None:
        ar = torch.arange(b, device=device, dtype=torch.int32)
        m = (torch.cat((ar, torch.roll(ar, -1))), torch.cat((ar, ar)))
        _MAPS[key] = m
    return m


class ImMatchNet(nn.Module):
    def __init__(self, feature_extraction_cnn: str = "resnet101", feature_extraction_last_layer: str = "",
                 feature_extraction_model_file: str | None = None, return_correlation: bool = False,
                 ncons_kernel_sizes=(3, 3, 3), ncons_channels=(10, 10, 1), normalize_features: bool = True,
                 train_fe: bool = False, use_cuda: bool = True, relocalization_k_size: int = 0,
                 half_precision: bool = False, checkpoint: str | None = None, dtype: str | None = None,
                 fold_bn: bool = True, corr_dtype: str | None = None, nc_precision: str = "bf16"):
        super().__init__()
        ck = None
        if checkpoint:
            ck = _load_reference_checkpoint(checkpoint)
            args = ck.get("args")
            if args is not None:
                ncons_channels = getattr(args, "ncons_channels", ncons_channels)
                ncons_kernel_sizes = getattr(args, "ncons_kernel_sizes", ncons_kernel_sizes)
        self.use_cuda = use_cuda and torch.cuda.is_available()
        self.normalize_features = normalize_features
        self.return_correlation = return_correlation
        self.relocalization_k_size = relocalization_k_size
        self.half_precision = half_precision
        # half_precision (the reference's eval_inloc.py setting, lib/model.py:253-267):
        # the reference halves AFTER its fp32 trunk and L2 norm, so do we -- IEEE-half
        # features, correlation, NeighConsensus input and hidden activation on the
        # f16 MFMA (the bf16 rate, 3 more mantissa bits), fp32 accumulation; the
        # trunk keeps bf16 (fp32's exponent range: unnormalised activations of a
        # deep trunk overflow fp16 -- measured on the random-init ResNet-101)
        if dtype is None:
            dtype = "bf16"
        if corr_dtype is None:
            corr_dtype = "fp16" if half_precision else "bf16"
        self.compute_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[dtype]
        self.fold_bn = fold_bn
        if corr_dtype not in ("bf16", "fp16", "fp8", "fp32"):
            raise ValueError("corr_dtype must be 'bf16', 'fp16', 'fp8' or 'fp32'")
        # fp8: OCP e4m3 correlation operands on the MX-fp8 MFMA and fp8
        # NeighConsensus (fp8 MFMA Conv4d) -- inference only.
        # fp32: fp32-accurate correlation + NeighConsensus (bf16x3 split on the
        # bf16 MFMA kernels), the reference's evaluation precision -- inference only
        self.corr_dtype = corr_dtype
        # nc_precision='fp32': NeighConsensus forward AND backward as bf16x3 splits
        # (fp32-accurate training at 3x the NC cost; ops/neigh_consensus.py NeighConsensusX3Fn)
        # nc_precision='mixed': the cheapest mix the per-stage ablation found to
        # train like 'fp32' (profiles/r5/ablation): fp32-accurate (bf16x3) trunk
        # and NeighConsensus forward, bf16 correlation and NeighConsensus backward
        if nc_precision not in ("bf16", "fp32", "mixed"):
            raise ValueError("nc_precision must be 'bf16', 'fp32' or 'mixed'")
        self.nc_precision = nc_precision
        if nc_precision in ("fp32", "mixed"):
            # fp32-accurate training: fp32 trunk, split (bf16x3) correlation when the
            # trunk is frozen, bf16x3 NeighConsensus forward and backward
            self.compute_dtype = torch.float32
        self.FeatureExtraction = FeatureExtraction(train_fe=train_fe, feature_extraction_cnn=feature_extraction_cnn,
                                                   feature_extraction_model_file=feature_extraction_model_file or "",
                                                   last_layer=feature_extraction_last_layer,
                                                   normalization=normalize_features, use_cuda=self.use_cuda)
        # fp32-accurate training runs its frozen trunk as bf16x3 splits (3x the bf16
        # MFMA work instead of MIOpen's fp32 convs at 1/16 of the bf16 rate); fp32
        # inference (corr_dtype='fp32', parity runs) keeps MIOpen's true fp32
        self.FeatureExtraction.fp32_trunk = "x3" if nc_precision in ("fp32", "mixed") else "miopen"
        self.FeatureCorrelation = FeatureCorrelation(shape="4D", normalization=False)
        self.NeighConsensus = NeighConsensus(use_cuda=self.use_cuda, kernel_sizes=list(ncons_kernel_sizes),
                                             channels=list(ncons_channels))
        if ck is not None:
            sd = ck["state_dict"]
            fe_sd = self.FeatureExtraction.state_dict()
            for name in fe_sd:
                if "num_batches_tracked" in name:
                    continue
                fe_sd[name].copy_(sd["FeatureExtraction." + name])
            for name, t in self.NeighConsensus.state_dict().items():
                t.copy_(sd["NeighConsensus." + name])
        self.FeatureExtraction.eval()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict, then drop the cross-call weight-pack cache
        (ops/packing.py): a load with ``assign=True`` rebinds the parameters and a
        later ``p.data`` edit would not bump their versions."""
        from ..ops.packing import clear_pack_cache
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        clear_pack_cache()
        return out

    # -- training-mode control: the backbone stays in eval (BN frozen), as in
    #    lib/model.py:251 and train.py:188.
    def train(self, mode: bool = True):
        super().train(mode)
        self.FeatureExtraction.eval()
        return self

    def _fe_dtype(self, x):
        return self.compute_dtype if x.is_cuda else None

    def extract(self, images: torch.Tensor) -> torch.Tensor:
        """images [N,3,H,W] -> L2-normalised packed features [N, H*W, C] (+ grid size)."""
        f = self.FeatureExtraction.trunk_forward(images, self._fe_dtype(images))
        if not self.FeatureExtraction.normalization:
            n, c, h, w = f.shape
            return f.permute(0, 2, 3, 1).reshape(n, h * w, c), (h, w)
        if self.corr_dtype == "fp8":
            if torch.is_grad_enabled() and self.training:
                raise RuntimeError("corr_dtype='fp8' is an inference path (no autograd)")
            return l2norm_pack_fp8(f), tuple(f.shape[-2:])
        if self.corr_dtype == "fp16" and not (torch.is_grad_enabled() and self.training):
            return l2norm_pack_f16(f), tuple(f.shape[-2:])
        if self.corr_dtype == "fp32" or self.nc_precision == "fp32":
            if f.requires_grad:
                if self.corr_dtype == "fp32":
                    raise RuntimeError("corr_dtype='fp32' is an inference path (no autograd)")
                return l2norm_pack(f), tuple(f.shape[-2:])     # trainable trunk: bf16 correlation operands
            return l2norm_pack_split(f), tuple(f.shape[-2:])
        return l2norm_pack(f), tuple(f.shape[-2:])

    def process_correlation(self, corr4d: torch.Tensor) -> torch.Tensor:
        """MutualMatching -> NeighConsensus -> MutualMatching (lib/model.py:274-276)."""
        self.NeighConsensus.fp8 = self.corr_dtype == "fp8"
        self.NeighConsensus.precision = ("fp32" if "fp32" in (self.corr_dtype, self.nc_precision)
                                         else "mixed" if self.nc_precision == "mixed" else "bf16")
        nc = self.NeighConsensus
        square = tuple(corr4d.shape[2:4]) == tuple(corr4d.shape[4:6])
        wrefs = [m.weight_ref() for m in nc.conv_layers()] if corr4d.is_cuda else []
        # the NC op's own path choice (ops/neigh_consensus.py select_path)
        path = (_nc_ops.select_path(corr4d, wrefs, nc.channels, nc.symmetric_mode, nc.fp8, nc.precision)
                if corr4d.is_cuda else "reference")
        f8 = path == "fused_fp8"
        if path in ("fused", "fused_fp8") and nc.symmetric_mode and square:
            # inference on the fused NC stack (bf16 / half, or e4m3 with
            # NCNET_NC_FP8 in fp8 mode): MutualMatching writes the 16-bit input
            # of both symmetric branches directly
            layers = nc.conv_layers()
            with segment("mutual_matching"):
                x2 = _mm_nc_input(corr4d, torch.float16 if self.corr_dtype == "fp16" else torch.bfloat16)
            biases = [m.bias if m.bias is not None else torch.zeros(m.out_channels, device=x2.device) for m in layers]
            _ext_count("nc_fused_k3_f8" if f8 else "nc_fused_k3")
            with segment("neigh_consensus"):
                fused = _nc_ops.neigh_consensus_fused_x2_fp8 if f8 else _nc_ops.neigh_consensus_fused_x2
                corr4d = fused(x2, wrefs, biases)
            with segment("mutual_matching"):
                return MutualMatching(corr4d)
        pks = nc.padded_input_ks(corr4d) if _ext_mod.use_hip(corr4d) else 0
        with segment("mutual_matching"):
            # training stack: MutualMatching also writes the NC input's padded planes
            xp = None
            if pks:
                corr4d, xp = _mm_padded(corr4d, pks)
            else:
                corr4d = MutualMatching(corr4d)
        with segment("neigh_consensus"):
            corr4d = self.NeighConsensus(corr4d, padded=xp)
        with segment("mutual_matching"):
            return MutualMatching(corr4d)

    def forward(self, tnf_batch):
        src, tgt = tnf_batch["source_image"], tnf_batch["target_image"]
        b = src.shape[0]
        if src.shape == tgt.shape:
            f, (h, w) = self.extract(torch.cat((src, tgt), 0))
            if isinstance(f, tuple):           # corr_dtype='fp32': (hi, lo) split operands
                fa, fb = (f[0][:b], f[1][:b]), (f[0][b:], f[1][b:])
            else:
                fa, fb = f[:b], f[b:]
            ha, wa, hb, wb = h, w, h, w
        else:
            fa, (ha, wa) = self.extract(src)
            fb, (hb, wb) = self.extract(tgt)
        return self.match_features(fa, (ha, wa), fb, (hb, wb))

    def match_features(self, fa, hwa, fb, hwb, packed_offsets: bool = False):
        """Everything after the backbone: correlation (+ k x k max-pool when
        relocalizing), MutualMatching, NeighConsensus, MutualMatching.  ``fa`` /
        ``fb`` come from ``extract`` -- eval_inloc.py extracts a query once and
        matches it against its 10 panos (the reference re-runs the query
        backbone per pano, eval_inloc.py:124-132; the features are identical).
        ``packed_offsets``: the k=2 max-pool offsets as one uint8 volume of 2-bit
        codes (decoded at the matched cells by eval/point_tnf.py) instead of
        four decoded volumes."""
        (ha, wa), (hb, wb) = hwa, hwb
        b = (fa[0] if isinstance(fa, tuple) else fa).shape[0]
        k = self.relocalization_k_size
        if isinstance(fa, tuple):
            corr4d = correlation_x3(fa, fb).view(b, 1, ha, wa, hb, wb)
            if k > 1:
                corr4d, delta = _maxpool4d(corr4d, k)
        elif k > 1:
            if k == 2 and ha % 2 == 0 and wa % 2 == 0 and hb % 2 == 0 and wb % 2 == 0:
                corr4d, delta = correlation_pool2(fa, fb, ha, wa, hb, wb, packed=packed_offsets)
            else:
                corr4d = correlation(fa, fb).view(b, 1, ha, wa, hb, wb)
                corr4d, delta = _maxpool4d(corr4d, k)
        else:
            corr4d = correlation(fa, fb).view(b, 1, ha, wa, hb, wb)
        corr4d = self.process_correlation(corr4d)
        if k > 1:
            return corr4d, delta
        return corr4d

    def weak_loss_volumes(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        """Positive and rolled-negative volumes [2B,1,h,w,h,w] for the weak loss.

        The negative pass of train.py:137 rolls the *source images* by -1; the
        backbone is in eval mode and acts per sample, so this equals rolling
        the source *features* -- the backbone runs once on 2B images instead
        of 4B."""
        b = src.shape[0]
        with segment("backbone"):
            f, hw = self.extract(torch.cat((src, tgt), 0))
        return self.weak_loss_volumes_from_features(f, hw, b)

    def weak_loss_volumes_from_features(self, f: torch.Tensor, hw, b: int) -> torch.Tensor:
        """``weak_loss_volumes`` after the backbone: ``f`` = extract() of the
        2B images [source; target] (engine/trainer.py TrunkPrefetcher runs it
        one step ahead on a side stream when the trunk is frozen)."""
        h, w = hw
        if isinstance(f, tuple):               # split operands (nc_precision / corr_dtype 'fp32')
            if _nc_ops.x3_dropped("corr"):     # precision ablation: bf16 correlation operands
                f = (f[0], torch.zeros_like(f[1]))
            amap, bmap = _pair_maps(b, f[0].device)
            with segment("correlation"):
                corr = correlation_x3((f[0][:b], f[1][:b]), (f[0][b:], f[1][b:]), amap, bmap)
            return self.process_correlation(corr.view(2 * b, 1, h, w, h, w))
        fa, fb = f[:b], f[b:]
        amap, bmap = _pair_maps(b, f.device)
        with segment("correlation"):
            corr = correlation(fa, fb, amap, bmap).view(2 * b, 1, h, w, h, w)
        return self.process_correlation(corr)
