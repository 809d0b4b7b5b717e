"""Single-layer Conv4d with the reference's API (lib/conv4d.py).

``conv4d(data, filters, bias=None, permute_filters=True, use_half=False)`` and
the ``Conv4d(in_channels, out_channels, kernel_size, bias=True,
pre_permuted_filters=True)`` module keep the reference's parameter names and
the pre-permuted ``[k, out, in, k, k, k]`` weight layout, so checkpoints
interchange (lib/conv4d.py:58-82).  The module is built
on ``nn.Module`` directly -- the reference's ``_ConvNd`` subclass no longer
constructs on modern torch.

On GPU the op runs the HIP implicit-GEMM kernels (forward, data gradient,
weight gradient); in the NC-Net model the fused stack in
``neigh_consensus.py`` is used instead of per-layer calls.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _ext
from . import reference as ref
from .neigh_consensus import _reduce_wgrad1, _reduce_wgrad16, wgrad16_partials, wgrad_groups
from .packing import pack_w16, pack_w1in, pack_w1out, transpose_for_dgrad


def _to_cl(x: torch.Tensor, c16: bool) -> torch.Tensor:
    """[N, C, I, J, K, L] -> channels-last bf16 ([N,I,J,K,L] if 1ch else padded to 16)."""
    n, c = x.shape[:2]
    if not c16:
        return x[:, 0].to(torch.bfloat16).contiguous()
    y = x.permute(0, 2, 3, 4, 5, 1)
    if c < 16:
        y = torch.nn.functional.pad(y, (0, 16 - c))
    return y.to(torch.bfloat16).contiguous()


def _from_cl(y: torch.Tensor, c: int) -> torch.Tensor:
    if y.dim() == 5:
        return y.unsqueeze(1)
    return y[..., :c].permute(0, 5, 1, 2, 3, 4)


def _conv_cl(xcl: torch.Tensor, w_std: torch.Tensor, cin: int, cout: int, mask=None) -> torch.Tensor:
    """Channels-last conv without bias; returns fp32/bf16 channels-last."""
    C = _ext.ext()
    ks = w_std.shape[-1]
    shp = xcl.shape[:5]
    if cin == 1:
        y = torch.empty(tuple(shp) + (16,), dtype=torch.bfloat16, device=xcl.device)
        C.conv1in_fwd(xcl, pack_w1in(w_std), None, mask, y, ks, 2 if mask is not None else 0)
    elif cout == 1:
        y = torch.empty(tuple(shp), dtype=torch.float32, device=xcl.device)
        C.conv1out_fwd(xcl, pack_w1out(w_std), None, y, ks, 0)
    else:
        y = torch.empty(tuple(shp) + (16,), dtype=torch.bfloat16, device=xcl.device)
        C.conv16_fwd(xcl, pack_w16(w_std), None, mask, y, ks, 2 if mask is not None else 0, 0)
    return y


def hip_supported(cin: int, cout: int, ks: int) -> bool:
    return ks in (3, 5) and cin <= 16 and cout <= 16 and not (cin == 1 and cout == 1)


class Conv4dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ref, bias):
        n, cin = x.shape[:2]
        cout = w_ref.shape[1]
        w_std = ref.conv4d_weight_to_std(w_ref).float()
        xcl = _to_cl(x, cin > 1)
        y = _conv_cl(xcl, w_std, cin, cout)
        out = _from_cl(y, cout).float()
        if bias is not None:
            out = out + bias.float().view(1, -1, 1, 1, 1, 1)
        ctx.save_for_backward(xcl, w_ref)
        ctx.meta = (cin, cout, bias is not None, x.dtype)
        return out.contiguous().to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        xcl, w_ref = ctx.saved_tensors
        cin, cout, has_bias, dt = ctx.meta
        C = _ext.ext()
        ks = w_ref.shape[0]
        w_std = ref.conv4d_weight_to_std(w_ref).float()
        gcl = _to_cl(g.float(), cout > 1)
        V, I, J, K, L = xcl.shape[:5]
        ng = wgrad_groups(ks, V * I * J * ((K + 24) // 25) * ((L + 24) // 25))
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            wt = transpose_for_dgrad(w_std)
            gx = _from_cl(_conv_cl(gcl, wt, cout, cin), cin).float().to(dt)
        if ctx.needs_input_grad[1]:
            if cin == 1:
                part = torch.empty((ng, ks * ks, ks * ks, 16), dtype=torch.float32, device=g.device)
                C.wgrad1(gcl, xcl, part, ks, 0, ng)
                dw = _reduce_wgrad1(part, ks, 0, cout)
            elif cout == 1:
                part = torch.empty((ng, ks * ks, ks * ks, 16), dtype=torch.float32, device=g.device)
                C.wgrad1(xcl, gcl, part, ks, 1, ng)
                dw = _reduce_wgrad1(part, ks, 1, cin)
            else:
                sw, _ = wgrad16_partials(C, xcl, gcl, ks, ng, False)
                dw = _reduce_wgrad16(sw, ks, cout, cin)
            gw = ref.conv4d_weight_from_std(dw).to(w_ref.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            gb = g.float().sum(dim=(0, 2, 3, 4, 5))
        return gx, gw, gb


def conv4d(data: torch.Tensor, filters: torch.Tensor, bias=None, permute_filters: bool = True,
           use_half: bool = False) -> torch.Tensor:
    """"Same"-padded 4D conv.  ``filters`` is ``[out, in, k, k, k, k]`` when
    ``permute_filters`` (as in lib/conv4d.py:16-17), else pre-permuted
    ``[k, out, in, k, k, k]``.  ``use_half`` is accepted for API parity; the
    GPU path always computes in bf16 with fp32 accumulation."""
    w_ref = ref.conv4d_weight_from_std(filters) if permute_filters else filters
    cin, cout, ks = w_ref.shape[2], w_ref.shape[1], w_ref.shape[0]
    if _ext.use_hip(data) and hip_supported(cin, cout, ks):
        return Conv4dFn.apply(data, w_ref, bias)
    return ref.conv4d(data, w_ref.to(data.dtype), None if bias is None else bias.to(data.dtype))


class Conv4d(nn.Module):
    """4D convolution, stride/dilation/groups = 1, "same" padding.

    Parameters: ``weight`` [k, out, in, k, k, k] (pre-permuted, the checkpoint
    layout) and ``bias`` [out]."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, bias: bool = True,
                 pre_permuted_filters: bool = True):
        super().__init__()
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, (k,) * 4
        self.stride, self.padding, self.dilation, self.groups = (1,) * 4, (0,) * 4, (1,) * 4, 1
        self.pre_permuted_filters = pre_permuted_filters
        w = torch.empty(out_channels, in_channels, k, k, k, k)
        # _ConvNd default init: kaiming_uniform(a=sqrt(5)) + uniform bias
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        if pre_permuted_filters:
            w = ref.conv4d_weight_from_std(w)
        self.weight = nn.Parameter(w)
        if bias:
            fan_in = in_channels * k ** 4
            bound = 1 / math.sqrt(fan_in)
            self.bias = nn.Parameter(torch.empty(out_channels).uniform_(-bound, bound))
        else:
            self.register_parameter("bias", None)
        self.use_half = False

    def weight_ref(self) -> torch.Tensor:
        """Weight in the pre-permuted checkpoint layout [k, out, in, k, k, k]."""
        return self.weight if self.pre_permuted_filters else ref.conv4d_weight_from_std(self.weight)

    def forward(self, x):
        return conv4d(x, self.weight, bias=self.bias, permute_filters=not self.pre_permuted_filters,
                      use_half=self.use_half)

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}"
