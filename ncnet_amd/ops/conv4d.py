"""Single-layer Conv4d with the reference's API (lib/conv4d.py).

``conv4d(data, filters, bias=None, permute_filters=True, use_half=False)`` and
the ``Conv4d(in_channels, out_channels, kernel_size, bias=True,
pre_permuted_filters=True)`` module keep the reference's parameter names and
the pre-permuted ``[k, out, in, k, k, k]`` weight layout, so checkpoints
interchange (lib/conv4d.py:58-82).  The module is built
on ``nn.Module`` directly -- the reference's ``_ConvNd`` subclass no longer
constructs on modern torch.

On GPU the op runs the HIP implicit-GEMM kernels (forward, data gradient,
weight gradient) through ``neigh_consensus.conv_layer`` -- the same
channel-blocked / ij-encoded layer path as the NC stack, so any channel
counts work; in the NC-Net model the fused stack in ``neigh_consensus.py``
is used instead of per-layer calls.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _ext
from . import reference as ref
from .neigh_consensus import HIP_KS, _layer_wgrad, blocks_to_ncl, conv_layer, planar_to_blocks
from .packing import ij_groups, transpose_for_dgrad


def _kind(cin: int, cout: int) -> str:
    return "11" if cin == 1 and cout == 1 else "1in" if cin == 1 else "1out" if cout == 1 else "16"


def _to_repr(x: torch.Tensor, c: int) -> torch.Tensor:
    """[N, C, I, J, K, L] -> the HIP layer representation: bf16 [N,I,J,K,L] (C = 1)
    or bf16 channels-last blocks [NB, N, I, J, K, L, 16]."""
    if c == 1:
        return x[:, 0].to(torch.bfloat16).contiguous()
    return planar_to_blocks(x.float().transpose(0, 1))


def _from_out(y: torch.Tensor, c: int) -> torch.Tensor:
    """conv_layer f32 output -> [N, C, I, J, K, L]."""
    return y.unsqueeze(1) if c == 1 else y.transpose(0, 1)


def hip_supported(cin: int, cout: int, ks: int) -> bool:
    return ks in HIP_KS and cin >= 1 and cout >= 1


class Conv4dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ref, bias):
        cin, cout = x.shape[1], w_ref.shape[1]
        w_std = ref.conv4d_weight_to_std(w_ref).float()
        h = _to_repr(x, cin)
        y = _from_out(conv_layer(h, w_std, cin, cout, bias=bias, relu=False, f32=True), cout)
        ctx.save_for_backward(h, w_ref)
        ctx.meta = (cin, cout, bias is not None, x.dtype)
        return y.contiguous().to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        h, w_ref = ctx.saved_tensors
        cin, cout, has_bias, dt = ctx.meta
        C = _ext.ext()
        ks = w_ref.shape[0]
        w_std = ref.conv4d_weight_to_std(w_ref).float()
        gr = _to_repr(g, cout)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _from_out(conv_layer(gr, transpose_for_dgrad(w_std), cout, cin, relu=False, f32=True), cin).to(dt)
        if ctx.needs_input_grad[1]:
            kind = _kind(cin, cout)
            xin = h
            if cin == 1:
                xin = torch.empty((ij_groups(ks),) + tuple(h.shape) + (16,), dtype=torch.bfloat16, device=h.device)
                C.ijpack(h, xin, ks, 1)
            gs = None
            if kind == "1out":
                gs = torch.empty((ij_groups(ks),) + tuple(gr.shape) + (16,), dtype=torch.bfloat16, device=h.device)
                C.ijpack(gr, gs, ks, -1)
            dw, _ = _layer_wgrad(C, kind, xin, gr, gs, ks, cin, cout)
            gw = ref.conv4d_weight_from_std(dw).to(w_ref.dtype)
        if has_bias and ctx.needs_input_grad[2]:
            gb = g.float().sum(dim=(0, 2, 3, 4, 5))
        return gx, gw, gb


def conv4d(data: torch.Tensor, filters: torch.Tensor, bias=None, permute_filters: bool = True,
           use_half: bool = False) -> torch.Tensor:
    """"Same"-padded 4D conv.  ``filters`` is ``[out, in, k, k, k, k]`` when
    ``permute_filters`` (as in lib/conv4d.py:16-17), else pre-permuted
    ``[k, out, in, k, k, k]``.  ``use_half`` is accepted for API parity; the
    GPU path always computes in bf16 with fp32 accumulation (any channel
    counts, kernel sizes 1/3/5/7; others raise unless
    NCNET_ALLOW_TORCH_FALLBACK=1)."""
    w_ref = ref.conv4d_weight_from_std(filters) if permute_filters else filters
    cin, cout, ks = w_ref.shape[2], w_ref.shape[1], w_ref.shape[0]
    if _ext.use_hip(data):
        if hip_supported(cin, cout, ks):
            _ext.count("conv4d_hip")
            return Conv4dFn.apply(data, w_ref, bias)
        _ext.torch_fallback(f"Conv4d kernel size {ks}")
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
