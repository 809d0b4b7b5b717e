"""Feature-extraction backbones, written in-repo (torchvision is not available).

Module names and ``nn.Sequential`` indices reproduce torchvision's, so the
state-dict keys match the reference checkpoints exactly:
``FeatureExtraction.model.{0,1,4,5,6}.*`` for the ResNet trunk that the
reference builds as ``Sequential([conv1, bn1, relu, maxpool, layer1, layer2,
layer3])`` (lib/model.py:37-44), VGG16 ``features[:pool4]`` (lib/model.py:24-35)
and DenseNet-201 ``features[:-4]`` (lib/model.py:69-74).

Weights are random-initialised (there is no network to fetch ImageNet weights);
a local state-dict is loaded strictly with ``load_trunk_state``.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F


def _kaiming(m: nn.Module):
    if isinstance(m, nn.Conv2d):
        nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.BatchNorm2d):
        nn.init.ones_(m.weight)
        nn.init.zeros_(m.bias)


class Bottleneck(nn.Module):
    """torchvision-v1.5 bottleneck (stride on the 3x3 conv)."""
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


class ResNet(nn.Module):
    """ResNet with torchvision attribute names (conv1, bn1, relu, maxpool, layer1..4)."""

    def __init__(self, layers=(3, 4, 23, 3)):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.apply(_kaiming)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * 4),
            )
        mods = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            mods.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*mods)


RESNET_LAYERS = ["conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4"]
RESNET_DEPTHS = {"resnet18": None, "resnet50": (3, 4, 6, 3), "resnet101": (3, 4, 23, 3), "resnet152": (3, 8, 36, 3)}


def resnet_trunk(arch: str = "resnet101", last_layer: str = "") -> nn.Sequential:
    """Sequential trunk up to ``last_layer`` (default layer3: stride 16, 1024 ch)."""
    depths = RESNET_DEPTHS.get(arch)
    if depths is None:
        raise ValueError(f"unsupported resnet variant {arch!r}")
    net = ResNet(depths)
    last = last_layer or "layer3"
    idx = RESNET_LAYERS.index(last)
    return nn.Sequential(*[getattr(net, n) for n in RESNET_LAYERS[: idx + 1]])


VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
VGG_LAYER_NAMES = ["conv1_1", "relu1_1", "conv1_2", "relu1_2", "pool1", "conv2_1", "relu2_1", "conv2_2",
                   "relu2_2", "pool2", "conv3_1", "relu3_1", "conv3_2", "relu3_2", "conv3_3", "relu3_3",
                   "pool3", "conv4_1", "relu4_1", "conv4_2", "relu4_2", "conv4_3", "relu4_3", "pool4",
                   "conv5_1", "relu5_1", "conv5_2", "relu5_2", "conv5_3", "relu5_3", "pool5"]


def vgg16_trunk(last_layer: str = "") -> nn.Sequential:
    """torchvision vgg16().features[: last_layer] (default pool4, stride 16, 512 ch)."""
    mods, c = [], 3
    for v in VGG16_CFG:
        if v == "M":
            mods.append(nn.MaxPool2d(2, 2))
        else:
            mods += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
            c = v
    last = last_layer or "pool4"
    idx = VGG_LAYER_NAMES.index(last)
    seq = nn.Sequential(*mods[: idx + 1])
    seq.apply(_kaiming)
    return seq


class _DenseLayer(nn.Module):
    def __init__(self, cin, growth, bn_size):
        super().__init__()
        self.norm1 = nn.BatchNorm2d(cin)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(cin, bn_size * growth, 1, bias=False)
        self.norm2 = nn.BatchNorm2d(bn_size * growth)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(bn_size * growth, growth, 3, padding=1, bias=False)

    def forward(self, feats):
        x = torch.cat(feats, 1) if isinstance(feats, (list, tuple)) else feats
        out = self.conv1(self.relu1(self.norm1(x)))
        return self.conv2(self.relu2(self.norm2(out)))


class _DenseBlock(nn.ModuleDict):
    def __init__(self, n, cin, growth, bn_size):
        super().__init__()
        for i in range(n):
            self.add_module("denselayer%d" % (i + 1), _DenseLayer(cin + i * growth, growth, bn_size))

    def forward(self, x):
        feats = [x]
        for layer in self.values():
            feats.append(layer(feats))
        return torch.cat(feats, 1)


class _Transition(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__()
        self.add_module("norm", nn.BatchNorm2d(cin))
        self.add_module("relu", nn.ReLU(inplace=True))
        self.add_module("conv", nn.Conv2d(cin, cout, 1, bias=False))
        self.add_module("pool", nn.AvgPool2d(2, 2))


def densenet201_trunk() -> nn.Sequential:
    """torchvision densenet201().features[:-4] (up to transition2, 256 ch, stride 16)."""
    growth, bn_size, blocks, c = 32, 4, (6, 12, 48, 32), 64
    feats = OrderedDict([
        ("conv0", nn.Conv2d(3, c, 7, stride=2, padding=3, bias=False)),
        ("norm0", nn.BatchNorm2d(c)),
        ("relu0", nn.ReLU(inplace=True)),
        ("pool0", nn.MaxPool2d(3, stride=2, padding=1)),
    ])
    for i, n in enumerate(blocks):
        feats["denseblock%d" % (i + 1)] = _DenseBlock(n, c, growth, bn_size)
        c = c + n * growth
        if i != len(blocks) - 1:
            feats["transition%d" % (i + 1)] = _Transition(c, c // 2)
            c = c // 2
    feats["norm5"] = nn.BatchNorm2d(c)
    full = nn.Sequential(feats)
    seq = nn.Sequential(*list(full.children())[:-4])
    seq.apply(_kaiming)
    return seq


DENSENET_FEATURES = ["conv0", "norm0", "relu0", "pool0", "denseblock1", "transition1", "denseblock2",
                     "transition2", "denseblock3", "transition3", "denseblock4", "norm5"]


def _trunk_key(key: str, cnn: str, n_mods: int) -> str | None:
    """Maps a full-model key (torchvision names: 'layer1.0.conv1.weight',
    'features.3.weight', 'features.denseblock1...') or a trunk key
    ('4.0.conv1.weight') to the trunk's key; None for a key of a layer past the
    truncation (layer4, fc, classifier, ...)."""
    for p in ("module.", "model."):
        if key.startswith(p):
            key = key[len(p):]
    head, _, rest = key.partition(".")
    if head.isdigit():
        return key if int(head) < n_mods else None
    if cnn.startswith("resnet"):
        if head == "fc":
            return None
        if head in RESNET_LAYERS:
            i = RESNET_LAYERS.index(head)
            return f"{i}.{rest}" if i < n_mods else None
        return key
    if head == "classifier":
        return None
    if head == "features":
        sub, _, rest2 = rest.partition(".")
        if cnn == "densenet201" and sub in DENSENET_FEATURES:
            i = DENSENET_FEATURES.index(sub)
        elif sub.isdigit():
            i = int(sub)
        else:
            return key
        return f"{i}.{rest2}" if i < n_mods else None
    return key


def load_trunk_state(trunk: nn.Sequential, sd: dict, cnn: str = "resnet101") -> None:
    """Strict load of a local state dict into a truncated trunk.

    The file may hold the trunk's own keys or the whole torchvision model's (the
    reference starts from ``models.resnet101(pretrained=True)`` and truncates,
    lib/model.py:37-44): keys of the layers past the truncation are dropped,
    and any trunk tensor the file does not fill, or any other key, raises an
    error that names them (never a silently half-initialised trunk)."""
    import re
    # torchvision's legacy densenet keys ('denselayer1.norm.1.weight' ->
    # 'denselayer1.norm1.weight'), as its densenet loader remaps them
    legacy = re.compile(r"^(.*denselayer\d+\.(?:norm|relu|conv))\.((?:[12])\.(?:weight|bias|running_mean|running_var))$")
    mapped, dropped = {}, 0
    for k, v in sd.items():
        m = legacy.match(k)
        if m:
            k = m.group(1) + m.group(2)
        tk = _trunk_key(k, cnn, len(trunk))
        if tk is None:
            dropped += 1
        else:
            mapped[tk] = v
    want = trunk.state_dict()
    # files older than BatchNorm's counter (the ImageNet checkpoints the
    # reference starts from) have no num_batches_tracked: 0, as BN's own loader
    for k in want:
        if k.endswith("num_batches_tracked") and k not in mapped:
            mapped[k] = torch.zeros_like(want[k])
    missing = sorted(set(want) - set(mapped))
    unexpected = sorted(set(mapped) - set(want))
    bad_shape = sorted(k for k in set(want) & set(mapped) if tuple(want[k].shape) != tuple(mapped[k].shape))
    if missing or unexpected or bad_shape:
        def few(xs):
            return ", ".join(xs[:8]) + (f" ... (+{len(xs) - 8})" if len(xs) > 8 else "")
        msg = [f"feature_extraction_model_file does not match the {cnn} trunk ({len(want)} tensors):"]
        if missing:
            msg.append(f"missing {len(missing)}: {few(missing)}")
        if unexpected:
            msg.append(f"unexpected {len(unexpected)}: {few(unexpected)}")
        if bad_shape:
            msg.append(f"shape mismatch {len(bad_shape)}: {few(bad_shape)}")
        raise RuntimeError("; ".join(msg))
    trunk.load_state_dict(mapped, strict=True)


def build_trunk(cnn: str = "resnet101", last_layer: str = "") -> tuple[nn.Sequential, int, int]:
    """Returns (trunk, out_channels, stride)."""
    if cnn == "vgg":
        return vgg16_trunk(last_layer), 512, 16
    if cnn.startswith("resnet") and not cnn.endswith("fpn"):
        last = last_layer or "layer3"
        ch = {"layer1": 256, "layer2": 512, "layer3": 1024, "layer4": 2048}.get(last, 64)
        stride = {"layer1": 4, "layer2": 8, "layer3": 16, "layer4": 32}.get(last, 4)
        return resnet_trunk(cnn, last), ch, stride
    if cnn == "densenet201":
        return densenet201_trunk(), 256, 16
    if cnn == "resnet101fpn":
        # lib/model.py:46-67 references an undefined fpn_body: unsupported there too.
        raise NotImplementedError("resnet101fpn is broken in the reference (undefined fpn_body, lib/model.py:61)")
    raise ValueError(f"unknown feature_extraction_cnn {cnn!r}")


@torch.no_grad()
def fold_frozen_bn(trunk: nn.Module) -> nn.Module:
    """Return a copy of an eval-mode trunk in which every Conv2d->BatchNorm2d
    pair is folded into a single biased conv (frozen BN is an affine map), so
    the frozen backbone issues one MIOpen conv per layer and no BN kernels."""
    import copy

    t = copy.deepcopy(trunk).eval()

    def fold(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride,
                          conv.padding, conv.dilation, conv.groups, bias=True).to(conv.weight.device)
        fused.weight.copy_(conv.weight * scale.view(-1, 1, 1, 1))
        b = conv.bias if conv.bias is not None else torch.zeros_like(bn.running_mean)
        fused.bias.copy_((b - bn.running_mean) * scale + bn.bias)
        return fused

    def walk(m: nn.Module):
        if isinstance(m, Bottleneck):
            m.conv1, m.bn1 = fold(m.conv1, m.bn1), nn.Identity()
            m.conv2, m.bn2 = fold(m.conv2, m.bn2), nn.Identity()
            m.conv3, m.bn3 = fold(m.conv3, m.bn3), nn.Identity()
            if m.downsample is not None:
                m.downsample = nn.Sequential(fold(m.downsample[0], m.downsample[1]))
            return
        if isinstance(m, nn.Sequential):
            kids = list(m._modules.items())
            for idx in range(len(kids) - 1):
                (na, a), (nb, b) = kids[idx], kids[idx + 1]
                if isinstance(a, nn.Conv2d) and isinstance(b, nn.BatchNorm2d):
                    m._modules[na] = fold(a, b)
                    m._modules[nb] = nn.Identity()
        for c in m.children():
            walk(c)

    walk(t)
    return t


# images per stem conv call of FrozenResNetPlan: the batch of train.py's default
# (16 pairs = 32 images), whose MIOpen solver choice the rounds' benches pinned
STEM_CHUNK = 32


# process-wide native / hipBLASLt choice per 1x1 conv shape (FrozenResNetPlan._c1)
_C1_CHOICE: dict = {}


class FrozenResNetPlan(nn.Module):
    """Inference plan of a frozen (BN-folded) ResNet trunk in one compute dtype.

    Built once from ``fold_frozen_bn(trunk)``; weights are cast and laid out up
    front (no per-step autocast casts).  Activations stay NHWC (channels-last)
    and each bottleneck runs as
      conv1 (1x1)  -> GEMM with bias+ReLU in the hipBLASLt epilogue
      conv2 (3x3)  -> MIOpen conv (no bias) + one fused bias+ReLU pass (HIP)
      conv3 (1x1)  -> GEMM with the residual as C operand (+ the downsample
                      GEMM/conv feeding it), then one fused bias+ReLU pass
    i.e. 2 activation round trips besides the convolutions, instead of ~7
    (MIOpen bias pass, ReLU, add, ReLU ...).  MIOpen's own fused
    conv+ReLU / conv+add+ReLU entry points were measured ~40x slower for bf16
    channels-last on MI355X (no fused solver), so they are not used.
    Reference: the frozen trunk of lib/model.py:37-44.
    """

    def __init__(self, folded: nn.Sequential, dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        self.dtype = dtype
        self.steps = []
        keep = []

        def w4(c: nn.Conv2d):
            w = c.weight.detach().to(dtype).contiguous(memory_format=torch.channels_last)
            keep.append(w)
            return w

        def wt(c: nn.Conv2d):  # 1x1 conv weight as the [Cin, Cout] GEMM operand (transposed view)
            w = c.weight.detach().to(dtype).reshape(c.out_channels, c.in_channels).contiguous()
            keep.append(w)
            return w.t()

        def bias(c: nn.Conv2d, dt):
            b = c.bias.detach().float() if c.bias is not None else torch.zeros(c.out_channels,
                                                                                 device=c.weight.device)
            return b.to(dt).contiguous()

        mods = list(folded.children())
        for idx, m in enumerate(mods):
            if isinstance(m, nn.Conv2d):
                relu = any(isinstance(n, nn.ReLU) for n in mods[idx + 1: idx + 3])
                self.steps.append(("conv", (w4(m), bias(m, torch.float32), m.stride, m.padding, relu)))
            elif isinstance(m, nn.MaxPool2d):
                self.steps.append(("maxpool", (m.kernel_size, m.stride, m.padding)))
            elif isinstance(m, nn.Sequential):
                for blk in m:
                    if not isinstance(blk, Bottleneck):
                        raise TypeError("FrozenResNetPlan expects Bottleneck layers")
                    b3 = bias(blk.conv3, torch.float32)
                    down = None
                    if blk.downsample is not None:
                        dc = blk.downsample[0]
                        b3 = b3 + bias(dc, torch.float32)   # relu(x W3 + b3 + (xs Wd + bd))
                        down = (wt(dc), 1) if dc.stride == (1, 1) else (w4(dc), dc.stride)
                    dn = None
                    if blk.downsample is not None:
                        dc = blk.downsample[0]
                        dn = (w4(dc), bias(dc, torch.float32), dc.stride[0], 0)
                    self.steps.append(("bottleneck", dict(
                        w1t=wt(blk.conv1), b1=bias(blk.conv1, dtype), w2=w4(blk.conv2),
                        b2=bias(blk.conv2, torch.float32), s2=blk.conv2.stride, w3t=wt(blk.conv3),
                        b3=b3.contiguous(), down=down,
                        # native NHWC implicit-GEMM kernels (csrc/conv2d.hip): every conv with its own bias
                        n1=(w4(blk.conv1), bias(blk.conv1, torch.float32), 1, 0),
                        n2=(w4(blk.conv2), bias(blk.conv2, torch.float32), blk.conv2.stride[0], 1),
                        n3=(w4(blk.conv3), bias(blk.conv3, torch.float32), 1, 0), nd=dn)))
            elif isinstance(m, (nn.ReLU, nn.Identity)):
                pass
            else:
                raise TypeError(f"FrozenResNetPlan: unsupported module {type(m).__name__}")
        self._keep = keep
        from .. import config as _config
        self.use_graphs = _config.RUNTIME.trunk_graph
        # "native": NHWC implicit-GEMM HIP kernels with fused bias/residual/ReLU
        # (csrc/conv2d.hip); "blas": hipBLASLt 1x1 GEMMs + MIOpen 3x3 + bias_act;
        # "auto" (default): native 3x3 / strided convs; every 1x1 stride-1 conv
        # (n1, the residual n3, the layer-1 downsample) on the native kernel or
        # on hipBLASLt with the same fused bias + residual + ReLU epilogue
        # (csrc/gemm_lt.hip), whichever measured faster for this input shape
        # (timed once per shape in the eager warm-up before the graph capture)
        self.conv_mode = _config.RUNTIME.trunk_conv
        self._graphs = {}
        self._tuned = {}

    @staticmethod
    def _bias_act(y: torch.Tensor, b: torch.Tensor, relu: bool) -> torch.Tensor:
        if y.is_cuda and y.dtype in (torch.bfloat16, torch.float16):
            from ..ops import _ext
            if _ext.use_hip(y):
                _ext.ext().bias_act_(y, b, 1 if relu else 0)
                return y
        shape = (1, -1, 1, 1) if y.dim() == 4 else (1, -1)
        y.add_(b.to(y.dtype).view(shape))
        return y.relu_() if relu else y

    @staticmethod
    def _pool_args(p):
        k, st, pad = p
        one = lambda v: v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)   # noqa: E731
        return one(k), one(st if st is not None else k), one(pad)

    def _pool_fusable(self, y: torch.Tensor, p) -> bool:
        if not (y.is_cuda and y.dtype in (torch.bfloat16, torch.float16) and y.shape[1] % 8 == 0):
            return False
        from ..ops import _ext
        k, st, pad = self._pool_args(p)
        return _ext.use_hip(y) and None not in (k, st, pad) and 2 * pad <= k

    def _maxpool_bias_act(self, y: torch.Tensor, b: torch.Tensor, p, relu: bool) -> torch.Tensor:
        from ..ops import _ext
        k, st, pad = self._pool_args(p)
        n, c, h, w = y.shape
        ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        out = torch.empty((n, c, ho, wo), dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
        _ext.ext().maxpool_bias_act(y, b.float().contiguous(), out, k, st, pad, 1 if relu else 0)
        return out

    def _stem_chunked(self, x, w, b, stride, pad, relu, pool):
        """The stem conv + fused bias / ReLU / max-pool over chunks of at most
        STEM_CHUNK images, into one channels-last output; None where the pool
        cannot be fused (the caller then runs the unchunked path)."""
        from ..ops import _ext
        k, st, pp = self._pool_args(pool)
        if None in (k, st, pp) or not (x.dtype in (torch.bfloat16, torch.float16) and w.shape[0] % 8 == 0
                                       and _ext.use_hip(x) and 2 * pp <= k):
            return None
        n = x.shape[0]
        bf = b.float().contiguous()
        out = None
        for c0 in range(0, n, STEM_CHUNK):
            y = F.conv2d(x[c0:c0 + STEM_CHUNK], w, None, stride, pad).contiguous(memory_format=torch.channels_last)
            if out is None:
                ho, wo = y.shape[-2:]
                out = torch.empty((n, y.shape[1], (ho + 2 * pp - k) // st + 1, (wo + 2 * pp - k) // st + 1),
                                  dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            _ext.ext().maxpool_bias_act(y, bf, out[c0:c0 + STEM_CHUNK], k, st, pp, 1 if relu else 0)
        return out

    @staticmethod
    def _nconv(x: torch.Tensor, p, relu: bool, res: torch.Tensor | None = None) -> torch.Tensor:
        from ..ops import _ext
        w, b, stride, pad = p
        n, _, h, wd = x.shape
        co, _, kh, kw = w.shape
        ho, wo = (h + 2 * pad - kh) // stride + 1, (wd + 2 * pad - kw) // stride + 1
        y = torch.empty((n, co, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        _ext.ext().conv2d_nhwc(x, w, b, res, y, stride, pad, 1 if relu else 0)
        return y

    @staticmethod
    def _rows(x: torch.Tensor) -> torch.Tensor:  # NCHW channels-last -> [N*H*W, C] view
        return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])

    @staticmethod
    def _nchw(y2d: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
        return y2d.view(n, h, w, -1).permute(0, 3, 1, 2)

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """GPU: replays a HIP graph of the whole trunk per input shape (captured
        after two eager warm-up runs, so MIOpen / hipBLASLt solver selection
        happens outside the capture).  At InLoc size the ~150 per-layer
        launches otherwise leave the GPU idle for a third of the trunk time."""
        if x.is_cuda and self.use_graphs:
            try:
                return self._graph_forward(x)
            except RuntimeError as err:          # capture unsupported -> stay eager
                self.use_graphs = False
                import warnings
                warnings.warn(f"FrozenResNetPlan: HIP graph capture disabled ({err})")
        return self._run(x)

    def _graph_forward(self, x: torch.Tensor) -> torch.Tensor:
        key = (tuple(x.shape), x.dtype, x.device)
        ent = self._graphs.get(key)
        if ent is None:
            # the graph input is already the plan's operand layout (16-bit,
            # channels-last): the per-call copy converts the images in one pass
            # instead of an fp32 copy followed by the conversion inside the graph
            static_in = torch.empty_like(x, dtype=self.dtype, memory_format=torch.channels_last)
            static_in.copy_(x)
            side = torch.cuda.Stream(device=x.device)
            side.wait_stream(torch.cuda.current_stream(x.device))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self._run(static_in)
            torch.cuda.current_stream(x.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                static_out = self._run(static_in)
            ent = (graph, static_in, static_out)
            self._graphs[key] = ent
        graph, static_in, static_out = ent
        static_in.copy_(x)
        graph.replay()
        return static_out.clone(memory_format=torch.channels_last)

    @staticmethod
    def _lt(x: torch.Tensor, p, relu: bool, res: torch.Tensor | None = None, tune: bool = False) -> torch.Tensor:
        """1x1 stride-1 conv as a hipBLASLt GEMM with the fused bias (+ residual)
        (+ ReLU) epilogue (csrc/gemm_lt.hip)."""
        from ..ops import _ext
        w, b = p[0], p[1]
        n, _, h, wd = x.shape
        y = torch.empty((n, w.shape[0], h, wd), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        _ext.ext().gemm_lt(x, w, b, res, y, 1 if relu else 0, 1 if tune else 0)
        return y

    def _c1(self, x: torch.Tensor, p, relu: bool, res: torch.Tensor | None, name) -> torch.Tensor:
        """A bottleneck conv (``name`` = (block, 'n1' | 'n3' | 'nd')): the native
        implicit-GEMM kernel or, for 1x1 stride-1 convs, hipBLASLt with the same
        fused epilogue, whichever measured faster at this input shape (timed in
        the eager warm-up before the graph capture; until then, and on a tie,
        native)."""
        w, _, stride, pad = p
        if not (w.shape[-1] == 1 and w.shape[-2] == 1 and stride == 1 and pad == 0):
            return self._nconv(x, p, relu, res)
        # one choice per (input shape, conv shape, epilogue) for the whole process:
        # every plan built in it (a fresh model, the volume-parallel slices) then
        # runs the same kernels on the same shapes, bit for bit
        key = (tuple(x.shape), x.dtype, tuple(w.shape), relu, res is not None)
        choice = _C1_CHOICE.get(key)
        if choice is None:
            if torch.cuda.is_current_stream_capturing():
                choice = "native"
            else:
                def t(fn):
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        fn()
                    e1.record()
                    e1.synchronize()
                    return e0.elapsed_time(e1)
                self._lt(x, p, relu, res, tune=True)          # hipBLASLt's candidates timed once per shape
                tn = t(lambda: self._nconv(x, p, relu, res))
                tb = t(lambda: self._lt(x, p, relu, res))
                choice = "blas" if tb < 0.97 * tn else "native"
                _C1_CHOICE[key] = choice
        self._tuned[(tuple(x.shape), name)] = choice
        return self._lt(x, p, relu, res) if choice == "blas" else self._nconv(x, p, relu, res)

    def tuned_choices(self) -> dict:
        """{(input shape, bottleneck index): 'native' | 'blas'} picked so far."""
        return dict(self._tuned)

    def _run(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.dtype).contiguous(memory_format=torch.channels_last)
        bi = -1
        fused_pool = False
        for si, (kind, p) in enumerate(self.steps):
            if kind == "bottleneck":
                bi += 1
            if kind == "conv":
                w, b, stride, pad, relu = p
                nxt = self.steps[si + 1] if si + 1 < len(self.steps) else None
                if nxt is not None and nxt[0] == "maxpool" and x.is_cuda and x.shape[0] > STEM_CHUNK:
                    # stem on MIOpen in fixed chunks of STEM_CHUNK images: its solver
                    # search at a large batch can settle on a naive kernel (a whole
                    # batch-256 step measured 1002 vs 306 ms in one of two runs);
                    # each chunk's bias + ReLU + max-pool writes its slice of the output
                    pooled = self._stem_chunked(x, w, b, stride, pad, relu, nxt[1])
                    if pooled is not None:
                        x, fused_pool = pooled, True
                        continue
                y = F.conv2d(x, w, None, stride, pad).contiguous(memory_format=torch.channels_last)
                if nxt is not None and nxt[0] == "maxpool" and self._pool_fusable(y, nxt[1]):
                    # stem: bias + ReLU + max-pool in one pass (csrc/epilogue.hip maxpool_bias_act)
                    x = self._maxpool_bias_act(y, b, nxt[1], relu)
                    fused_pool = True
                else:
                    x = self._bias_act(y, b, relu)
            elif kind == "maxpool":
                if fused_pool:
                    fused_pool = False
                else:
                    x = F.max_pool2d(x, *p).contiguous(memory_format=torch.channels_last)
            elif self.conv_mode in ("native", "auto") and x.is_cuda and self.dtype in (torch.bfloat16, torch.float16):
                if self.conv_mode == "auto":
                    y1 = self._c1(x, p["n1"], True, None, (bi, "n1"))
                    y2 = self._nconv(y1, p["n2"], True)
                    idt = x if p["nd"] is None else self._c1(x, p["nd"], False, None, (bi, "nd"))
                    x = self._c1(y2, p["n3"], True, idt, (bi, "n3"))
                else:
                    y1 = self._nconv(x, p["n1"], True)
                    y2 = self._nconv(y1, p["n2"], True)
                    idt = x if p["nd"] is None else self._nconv(x, p["nd"], False)
                    x = self._nconv(y2, p["n3"], True, idt)
            else:
                n, _, h, w = x.shape
                x2d = self._rows(x)
                y1 = torch._addmm_activation(p["b1"], x2d, p["w1t"])            # relu(x W1 + b1)
                y2 = F.conv2d(self._nchw(y1, n, h, w), p["w2"], None, p["s2"], 1)
                y2 = self._bias_act(y2.contiguous(memory_format=torch.channels_last), p["b2"], True)
                n2, _, h2, w2 = y2.shape
                if p["down"] is None:
                    idt = x2d
                elif p["down"][1] == 1:
                    idt = torch.mm(x2d, p["down"][0])
                else:
                    idt = self._rows(F.conv2d(x, p["down"][0], None, p["down"][1]).contiguous(
                        memory_format=torch.channels_last))
                out = torch.addmm(idt, self._rows(y2), p["w3t"])                # x W3 + identity
                x = self._nchw(self._bias_act(out, p["b3"], True), n2, h2, w2)
        return x


class FrozenResNetPlanX3(nn.Module):
    """fp32-accurate plan of a frozen (BN-folded) ResNet trunk on the bf16
    matrix cores: the "bf16x3" split of every conv (the reference runs the
    trunk in fp32, lib/model.py:84; ``ImMatchNet(nc_precision='fp32')``).

    Activations are [N, H, W, 2C] bf16 holding hi = bf16(x) and lo = bf16(x -
    hi) (x to ~2^-16 relative); every conv is conv2d_nhwc_v3's X3 mode
    (csrc/conv2d.hip: acc = X_hi W_hi + X_lo W_hi + X_hi W_lo in fp32, bias,
    the hi + lo residual and ReLU in fp32, output split again), the 7x7 stem a
    GEMM over an im2col of the fp32 image (K = 147 padded to 192), the stem
    max-pool compares hi + lo.  Three bf16 MFMA passes per conv instead of the
    MIOpen fp32 implicit GEMMs (1/16 of the bf16 rate on CDNA4); the output
    is fp32 NCHW (channels-last).  The whole trunk replays as one HIP graph
    per input shape.
    """

    KP_ALIGN = 64

    def __init__(self, folded: nn.Sequential):
        super().__init__()
        self.steps = []

        def split3(w_cl: torch.Tensor) -> torch.Tensor:
            """[Cout, ..., Cin] fp32 -> [Cout, ..., 3 Cin] bf16 = [W_hi | W_hi | W_lo]."""
            hi = w_cl.to(torch.bfloat16)
            lo = (w_cl - hi.float()).to(torch.bfloat16)
            return torch.cat((hi, hi, lo), -1).contiguous()

        def conv_w(c: nn.Conv2d) -> torch.Tensor:
            return split3(c.weight.detach().float().permute(0, 2, 3, 1))      # [Cout, KH, KW, 3 Cin]

        def bias(c: nn.Conv2d) -> torch.Tensor:
            if c.bias is None:
                return torch.zeros(c.out_channels, device=c.weight.device)
            return c.bias.detach().float().contiguous()

        mods = list(folded.children())
        for idx, m in enumerate(mods):
            if isinstance(m, nn.Conv2d):
                relu = any(isinstance(n, nn.ReLU) for n in mods[idx + 1: idx + 3])
                co, ci, kh, kw = m.weight.shape
                k = kh * kw * ci
                kp = -(-k // self.KP_ALIGN) * self.KP_ALIGN
                w = m.weight.detach().float().permute(0, 2, 3, 1).reshape(co, k)
                w = torch.cat((w, w.new_zeros(co, kp - k)), 1)
                self.steps.append(("stem", dict(w3=split3(w).reshape(co, 1, 1, 3 * kp), b=bias(m), kh=kh, kw=kw,
                                                stride=m.stride[0], pad=m.padding[0], kp=kp, relu=relu)))
            elif isinstance(m, nn.MaxPool2d):
                k, st, pad = FrozenResNetPlan._pool_args((m.kernel_size, m.stride, m.padding))
                self.steps.append(("maxpool", (k, st, pad)))
            elif isinstance(m, nn.Sequential):
                for blk in m:
                    if not isinstance(blk, Bottleneck):
                        raise TypeError("FrozenResNetPlanX3 expects Bottleneck layers")
                    dn = None
                    if blk.downsample is not None:
                        dc = blk.downsample[0]
                        dn = (conv_w(dc), bias(dc), dc.stride[0], 0)
                    self.steps.append(("bottleneck", dict(
                        n1=(conv_w(blk.conv1), bias(blk.conv1), 1, 0),
                        n2=(conv_w(blk.conv2), bias(blk.conv2), blk.conv2.stride[0], 1),
                        n3=(conv_w(blk.conv3), bias(blk.conv3), 1, 0), nd=dn)))
            elif isinstance(m, (nn.ReLU, nn.Identity)):
                pass
            else:
                raise TypeError(f"FrozenResNetPlanX3: unsupported module {type(m).__name__}")
        from .. import config as _config
        self.use_graphs = _config.RUNTIME.trunk_graph
        self._graphs = {}

    @staticmethod
    def _conv(x: torch.Tensor, p, relu: bool, res: torch.Tensor | None = None) -> torch.Tensor:
        from ..ops import _ext
        w3, b, stride, pad = p
        n, h, wd, _ = x.shape
        co, kh, kw, _ = w3.shape
        ho, wo = (h + 2 * pad - kh) // stride + 1, (wd + 2 * pad - kw) // stride + 1
        y = torch.empty((n, ho, wo, 2 * co), dtype=torch.bfloat16, device=x.device)
        _ext.ext().conv2d_nhwc_x3(x, w3, b, res, y, stride, pad, 1 if relu else 0)
        return y

    def _run(self, img: torch.Tensor) -> torch.Tensor:
        from ..ops import _ext
        C = _ext.ext()
        x = img.float().contiguous(memory_format=torch.channels_last)
        for kind, p in self.steps:
            if kind == "stem":
                n, _, h, w = x.shape
                ho = (h + 2 * p["pad"] - p["kh"]) // p["stride"] + 1
                wo = (w + 2 * p["pad"] - p["kw"]) // p["stride"] + 1
                a = torch.empty((n * ho * wo, 2 * p["kp"]), dtype=torch.bfloat16, device=x.device)
                C.stem_im2col_x3(x, a, p["kh"], p["kw"], p["stride"], p["pad"])
                x = self._conv(a.view(n, ho, wo, 2 * p["kp"]), (p["w3"], p["b"], 1, 0), p["relu"])
            elif kind == "maxpool":
                k, st, pad = p
                n, h, w, c2 = x.shape
                y = torch.empty((n, (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1, c2),
                                dtype=torch.bfloat16, device=x.device)
                C.maxpool_x3(x, y, k, st, pad)
                x = y
            else:
                y1 = self._conv(x, p["n1"], True)
                y2 = self._conv(y1, p["n2"], True)
                idt = x if p["nd"] is None else self._conv(x, p["nd"], False)
                x = self._conv(y2, p["n3"], True, idt)
        n, h, w, c2 = x.shape
        out = torch.empty((n, h, w, c2 // 2), dtype=torch.float32, device=x.device)
        C.x3_to_f32(x, out)
        return out.permute(0, 3, 1, 2)          # NCHW view, channels-last memory

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.use_graphs:
            return self._run(x)
        key = (tuple(x.shape), x.dtype, x.device)
        ent = self._graphs.get(key)
        if ent is None:
            try:
                static_in = x.clone()
                side = torch.cuda.Stream(device=x.device)
                side.wait_stream(torch.cuda.current_stream(x.device))
                with torch.cuda.stream(side):
                    self._run(static_in)
                torch.cuda.current_stream(x.device).wait_stream(side)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    static_out = self._run(static_in)
            except RuntimeError as err:            # capture unsupported -> stay eager (loudly)
                import warnings
                warnings.warn(f"FrozenResNetPlanX3: HIP graph capture disabled ({err})")
                self.use_graphs = False
                return self._run(x)
            ent = self._graphs[key] = (graph, static_in, static_out)
        graph, static_in, static_out = ent
        static_in.copy_(x)
        graph.replay()
        return static_out.clone(memory_format=torch.channels_last)
