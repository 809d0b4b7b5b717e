"""Probe: bf16x3 NC training gradients (fused and per-conv paths) against the
fp64 oracle computed on the CPU and on the GPU."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from ncnet_amd.ops import reference as ref  # noqa: E402
from ncnet_amd.ops.neigh_consensus import NeighConsensusX3Fn, NeighConsensusX3FusedFn, layer_kinds  # noqa: E402
from tests.test_gpu_x3 import _params, rl2  # noqa: E402


def grads(fn, x, ws, bs, gy):
    for p in ws + bs:
        p.grad = None
    y = fn(x)
    (y * gy).sum().backward()
    out = [y.detach()]
    for w, b in zip(ws, bs):
        out += [w.grad.clone(), b.grad.clone()]
    return out


def main():
    ks, ch = (5, 5, 5), (16, 16, 1)
    shape = (2, 1, 9, 7, 9, 7) if len(sys.argv) < 2 else tuple(int(v) for v in sys.argv[1:])
    ws, bs = _params(ks, ch, 11)
    torch.manual_seed(7)
    x = torch.rand(shape, device="cuda")
    kinds = tuple(layer_kinds(list(ch), list(ks)))
    params = []
    for w, b in zip(ws, bs):
        params += [w, b]
    y0 = NeighConsensusX3FusedFn.apply(x, kinds, ch, *params)
    gy = torch.randn_like(y0)
    fused = grads(lambda t: NeighConsensusX3FusedFn.apply(t, kinds, ch, *params), x, ws, bs, gy)
    old = grads(lambda t: NeighConsensusX3Fn.apply(t, True, kinds, ch, *params), x, ws, bs, gy)
    for dev in ("cuda", "cpu"):
        wd = [w.detach().double().to(dev).requires_grad_(True) for w in ws]
        bd = [b.detach().double().to(dev).requires_grad_(True) for b in bs]
        yr = ref.neigh_consensus(x.double().to(dev), wd, bd, True)
        (yr * gy.double().to(dev)).sum().backward()
        want = [yr.detach()]
        for w, b in zip(wd, bd):
            want += [w.grad, b.grad]
        for name, got in (("fused", fused), ("old", old)):
            print(dev, name, ["%.1e" % rl2(a.cpu(), b.cpu()) for a, b in zip(got, want)], flush=True)
    print("fused vs old", ["%.1e" % rl2(a, b) for a, b in zip(fused, old)], flush=True)


if __name__ == "__main__":
    main()
