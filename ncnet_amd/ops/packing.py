"""Repack Conv4d weights into the MFMA fragment order each HIP kernel reads.

Weights arrive in the standard layout ``[Cout, Cin, k, k, k, k]`` (see
``reference.conv4d_weight_to_std`` for the checkpoint's pre-permuted layout).
Packing is a single gather with cached index tensors, done once per forward
(the tensors are <= 320 KB), in bf16.

* ``pack_w16``   Cin=16, Cout=16 -> [k*k, ceil(k*k/2), 64, 8]
                 lane l of pair q: W[co=l&15, ci=8((l>>4)&1)+j, di, dj, tap=2q+(l>>5)]
* ``pack_w1in``  Cin=1,  Cout=16 -> [k*k, ceil(k/4), 64, 8]
                 lane l of MFMA m: W[co=l&15, 0, di, dj, dk=4m+(l>>4), dl=j]
* ``pack_w1out`` Cin=16, Cout=1  -> [k*k, ceil((k+3)^2/2), 64, 8]
                 lane l of pair p: W'[tau=2p+(l>>5), s=l&15] for ci=8((l>>4)&1)+j
                 with W'[tau, s] = W[0, ci, di, dj, tau - s] (4x4 shift grid)

``transpose_for_dgrad`` gives the weights of the data-gradient convolution
(swap in/out channels, flip all four kernel axes).
"""
from __future__ import annotations

import functools

import torch


def transpose_for_dgrad(w_std: torch.Tensor) -> torch.Tensor:
    return w_std.transpose(0, 1).flip(2, 3, 4, 5)


@functools.lru_cache(maxsize=None)
def _idx16(ks: int):
    nt = ks * ks
    nq = (nt + 1) // 2
    q = torch.arange(nq).view(nq, 1, 1)
    lane = torch.arange(64).view(1, 64, 1)
    j = torch.arange(8).view(1, 1, 8)
    tap = 2 * q + (lane >> 5)
    co = (lane & 15).expand(nq, 64, 8)
    ci = (8 * ((lane >> 4) & 1) + j).expand(nq, 64, 8)
    valid = (tap < nt).expand(nq, 64, 8)
    tap = torch.clamp(tap, max=nt - 1).expand(nq, 64, 8)
    return co, ci, tap, valid


@functools.lru_cache(maxsize=None)
def _idx1in(ks: int):
    nm = (ks + 3) // 4
    m = torch.arange(nm).view(nm, 1, 1)
    lane = torch.arange(64).view(1, 64, 1)
    j = torch.arange(8).view(1, 1, 8)
    dk = 4 * m + (lane >> 4)
    dl = j
    valid = ((dk < ks) & (dl < ks)).expand(nm, 64, 8)
    tap = (torch.clamp(dk, max=ks - 1) * ks + torch.clamp(dl, max=ks - 1)).expand(nm, 64, 8)
    co = (lane & 15).expand(nm, 64, 8)
    return co, tap, valid


@functools.lru_cache(maxsize=None)
def _idx1out(ks: int):
    ts = ks + 3
    npair = (ts * ts + 1) // 2
    p = torch.arange(npair).view(npair, 1, 1)
    lane = torch.arange(64).view(1, 64, 1)
    j = torch.arange(8).view(1, 1, 8)
    tau = 2 * p + (lane >> 5)
    s = lane & 15
    sk, sl = s // 4, s % 4
    tk, tl = tau // ts, tau % ts
    dk, dl = tk - sk, tl - sl
    valid = ((tau < ts * ts) & (dk >= 0) & (dk < ks) & (dl >= 0) & (dl < ks)).expand(npair, 64, 8)
    tap = (torch.clamp(dk, 0, ks - 1) * ks + torch.clamp(dl, 0, ks - 1)).expand(npair, 64, 8)
    ci = (8 * ((lane >> 4) & 1) + j).expand(npair, 64, 8)
    return ci, tap, valid


def _as_std(w_std: torch.Tensor, cout: int, cin: int) -> torch.Tensor:
    """Zero-pad [co, ci, k^4] channels up to (cout, cin)."""
    co, ci = w_std.shape[:2]
    if co == cout and ci == cin:
        return w_std
    out = w_std.new_zeros((cout, cin) + tuple(w_std.shape[2:]))
    out[:co, :ci] = w_std
    return out


def pack_w16(w_std: torch.Tensor) -> torch.Tensor:
    ks = w_std.shape[-1]
    w = _as_std(w_std, 16, 16).reshape(16, 16, ks * ks, ks * ks)
    co, ci, tap, valid = (t.to(w.device) for t in _idx16(ks))
    vals = w[co, ci, :, tap]                      # [nq, 64, 8, k*k]
    vals = vals * valid.unsqueeze(-1).to(vals.dtype)
    return vals.permute(3, 0, 1, 2).contiguous().to(torch.bfloat16)


def pack_w1in(w_std: torch.Tensor) -> torch.Tensor:
    ks = w_std.shape[-1]
    assert w_std.shape[1] == 1
    w = _as_std(w_std, 16, 1).reshape(16, ks * ks, ks * ks)
    co, tap, valid = (t.to(w.device) for t in _idx1in(ks))
    vals = w[co, :, tap]                           # [nm, 64, 8, k*k]
    vals = vals * valid.unsqueeze(-1).to(vals.dtype)
    return vals.permute(3, 0, 1, 2).contiguous().to(torch.bfloat16)


def pack_w1out(w_std: torch.Tensor) -> torch.Tensor:
    ks = w_std.shape[-1]
    assert w_std.shape[0] == 1
    w = _as_std(w_std, 1, 16).reshape(16, ks * ks, ks * ks)
    ci, tap, valid = (t.to(w.device) for t in _idx1out(ks))
    vals = w[ci, :, tap]                           # [npair, 64, 8, k*k]
    vals = vals * valid.unsqueeze(-1).to(vals.dtype)
    return vals.permute(3, 0, 1, 2).contiguous().to(torch.bfloat16)


# ---------------------------------------------------------------------------
# j-offset <-> channel encoding of the 1-channel layers (see csrc/jshift.hip).
# A Cin=1 layer W1 [co,1,k^4] becomes a 16->16 conv over jpack(X0) whose kernel
# lives on the dj=P plane only; a Cout=1 layer W3 [1,ci,k^4] becomes a 16->16
# conv (channels = dj) followed by jsum.

def jc_in_weights(w_std: torch.Tensor) -> torch.Tensor:
    """[co, 1, k^4] -> [16, 16, k^4]: out[co][c][di][P][dk][dl] = w[co][0][di][c][dk][dl]."""
    co, ks = w_std.shape[0], w_std.shape[-1]
    out = w_std.new_zeros((16, 16) + (ks,) * 4)
    out[:co, :ks, :, ks // 2] = w_std[:, 0].permute(0, 2, 1, 3, 4)
    return out


def jc_out_weights(w_std: torch.Tensor) -> torch.Tensor:
    """[1, ci, k^4] -> [16, 16, k^4]: out[c][ci][di][P][dk][dl] = w[0][ci][di][c][dk][dl]."""
    ci, ks = w_std.shape[1], w_std.shape[-1]
    out = w_std.new_zeros((16, 16) + (ks,) * 4)
    out[:ks, :ci, :, ks // 2] = w_std[0].permute(2, 0, 1, 3, 4)
    return out


def jc_in_grad(s5: torch.Tensor, cout: int) -> torch.Tensor:
    """dW of the dj=P slice [co, c, di, dk, dl] -> [co, 1, di, dj=c, dk, dl]."""
    ks = s5.shape[-1]
    return s5[:cout, :ks].permute(0, 2, 1, 3, 4).unsqueeze(1).contiguous()


def jc_out_grad(s5: torch.Tensor, cin: int) -> torch.Tensor:
    """dW of the dj=P slice [c, ci, di, dk, dl] -> [1, ci, di, dj=c, dk, dl]."""
    ks = s5.shape[-1]
    return s5[:ks, :cin].permute(1, 2, 0, 3, 4).unsqueeze(0).contiguous()


# ---------------------------------------------------------------------------
# ij encoding (csrc/jshift.hip ijpack / ijsum): both plane offsets (di, dj) go
# into channels, combo q = di*k + dj, 16 combos per group, G = ceil(k*k/16).
# A Cin=1 layer becomes sum_g conv2d_(dk,dl)(ijpack(X0)[g], W_g) and a Cout=1
# layer ijsum(conv2d_(dk,dl)(X, W_g) for each g), all on conv16's group-plane
# mode; plane weights are [G, 16 out, 16 in, k, k].

def ij_groups(ks: int) -> int:
    return (ks * ks + 15) // 16


def pack_w16_planes(wp: torch.Tensor) -> torch.Tensor:
    """[NPL, 16 co, 16 ci, k, k] -> [NPL, ceil(k*k/2), 64, 8] (pack_w16 per plane)."""
    npl, ks = wp.shape[0], wp.shape[-1]
    w = wp.reshape(npl, 16, 16, ks * ks)
    co, ci, tap, valid = (t.to(w.device) for t in _idx16(ks))
    vals = w[:, co, ci, tap] * valid.to(w.dtype)      # [npl, nq, 64, 8]
    return vals.contiguous().to(torch.bfloat16)


def ij_in_weights(w_std: torch.Tensor) -> torch.Tensor:
    """[co, 1, k^4] -> [G, 16 co, 16 c, k, k]: out[g][co][c] = w[co][0][di][dj] with 16g + c = di*k + dj."""
    co, ks = w_std.shape[0], w_std.shape[-1]
    G = ij_groups(ks)
    tmp = w_std.new_zeros((16, G * 16, ks, ks))
    tmp[:co, : ks * ks] = w_std[:, 0].reshape(co, ks * ks, ks, ks)
    return tmp.view(16, G, 16, ks, ks).permute(1, 0, 2, 3, 4).contiguous()


def ij_out_weights(w_std: torch.Tensor) -> torch.Tensor:
    """[1, ci, k^4] -> [G, 16 c, 16 ci, k, k]: out[g][c][ci] = w[0][ci][di][dj] with 16g + c = di*k + dj."""
    ci, ks = w_std.shape[1], w_std.shape[-1]
    G = ij_groups(ks)
    tmp = w_std.new_zeros((G * 16, 16, ks, ks))
    tmp[: ks * ks, :ci] = w_std[0].reshape(ci, ks * ks, ks, ks).permute(1, 0, 2, 3)
    return tmp.view(G, 16, 16, ks, ks).contiguous()


def plane_dgrad_weights(wp: torch.Tensor) -> torch.Tensor:
    """Data-gradient weights of a (dk, dl)-only plane conv: swap channels, flip taps."""
    return wp.transpose(1, 2).flip(-2, -1)


def ij_in_grad(s: torch.Tensor, cout: int) -> torch.Tensor:
    """s [G, tap, c, co] (plane wgrad of X = ijpack(X0)[g], G = grad) -> dW [co, 1, k, k, k, k]."""
    G, nt = s.shape[0], s.shape[1]
    ks = int(round(nt ** 0.5))
    d = s.permute(3, 0, 2, 1).reshape(16, G * 16, nt)[:cout, :nt]      # [co, q, tap]
    return d.reshape(cout, 1, ks, ks, ks, ks).contiguous()


def ij_out_grad(s: torch.Tensor, cin: int) -> torch.Tensor:
    """s [G, tap, ci, c] (plane wgrad of X = layer input, G = ijpack(g, -1)[g]) -> dW [1, ci, k, k, k, k]."""
    G, nt = s.shape[0], s.shape[1]
    ks = int(round(nt ** 0.5))
    d = s.permute(2, 0, 3, 1).reshape(16, G * 16, nt)[:cin, :nt]      # [ci, q, tap]
    return d.reshape(1, cin, ks, ks, ks, ks).contiguous()


# ---------------------------------------------------------------------------
# kl kernels (csrc/conv4d_kl.hip): in-plane (dk, dl) shifts resolved in LDS.

def pack_kl_in(w_std: torch.Tensor) -> torch.Tensor:
    """Cin=1 -> Cout<=16 weights [co, 1, k, k, k, k] -> [ceil(k^4/32), 64, 8] bf16.

    Lane l of K step s holds W[co=l&15, tap=32s+8(l>>4)+j] with the taps in
    (di, dj, dk, dl) row-major order (zero past k^4 and for co >= Cout)."""
    cout, ks = w_std.shape[0], w_std.shape[2]
    nk = ks ** 4
    ns = (nk + 31) // 32
    wf = w_std.new_zeros((16, ns * 32), dtype=torch.float32)
    wf[:cout, :nk] = w_std.reshape(cout, nk).float()
    return wf.reshape(16, ns, 4, 8).permute(1, 2, 0, 3).reshape(ns, 64, 8).to(torch.bfloat16).contiguous()


def kl_dgrad_in_weights(w_std: torch.Tensor) -> torch.Tensor:
    """Data gradient of a Cout=1 layer as a 1 -> Cin conv: [1, ci, k^4] -> [ci, 1, k^4 flipped]."""
    return transpose_for_dgrad(w_std)


def pack_kl_out(w_std: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """Cin<=16 -> Cout=1 weights [1, ci, k, k, k, k] -> [k*k + 1, ceil(k*k/16), 16, 16].

    Entry [p=(di,dj), ct, r, c] = W[0, c, di, dj, dk, dl] for the in-plane combo
    16*ct + r = dk*k + dl (zero past k*k, for c >= Cin and on the extra
    all-zero plane k*k used to pad odd plane counts)."""
    cin, ks = w_std.shape[1], w_std.shape[2]
    nt = ks * ks
    nct = (nt + 15) // 16
    out = w_std.new_zeros((nt + 1, nct * 16, 16), dtype=torch.float32)
    out[:nt, :nt, :cin] = w_std[0].float().permute(1, 2, 3, 4, 0).reshape(nt, nt, cin)
    return out.reshape(nt + 1, nct, 16, 16).to(dtype).contiguous()
