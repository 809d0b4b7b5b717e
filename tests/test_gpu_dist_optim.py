"""GPU: the RCCL process group really forms and every collective the
framework issues is verified over it (world size 1 under torchrun on the
one-GPU box), and the HIP FlatAdam kernels match
torch.optim.Adam and skip non-finite steps exactly."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives(tmp_path):
    out = os.path.join(ROOT, "gpurun_out", "rccl_check.json")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29547", os.path.join(ROOT, "scripts", "rccl_check.py"),
           "--out", out]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["comm"]["backend"] == "nccl" and res["comm"]["process_group"], res
    assert res["comm"].get("rccl_version"), res
    assert res["all_ok"], res


def _params(dev):
    g = torch.Generator().manual_seed(0)
    shapes = [(5, 16, 16, 5, 5, 5), (16,), (5, 1, 16, 5, 5, 5), (1,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]


def _grads(ps, step):
    g = torch.Generator().manual_seed(1000 + step)
    return [torch.randn(p.shape, generator=g).to(p.device) for p in ps]


def test_flat_adam_hip_matches_torch_adam():
    from ncnet_amd.engine.optim import FlatAdam
    from ncnet_amd.ops import _ext
    pa, pb = _params("cuda"), _params("cuda")
    ta = torch.optim.Adam(pa, lr=5e-4)
    fb = FlatAdam(pb, lr=5e-4)
    assert fb._hip and _ext.available()
    for step in range(8):
        ta.zero_grad()
        fb.zero_grad()
        for p, q, g in zip(pa, pb, _grads(pa, step)):
            p.grad = g.clone()
            q.grad.copy_(g)
        fb.mark_loss(torch.tensor(0.5, device="cuda"))
        ta.step()
        fb.step()
    torch.cuda.synchronize()
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=2e-6, atol=1e-7)
    assert fb.steps_taken == 8 and fb.skipped_steps == 0


@pytest.mark.parametrize("bad", ["grad", "loss"])
def test_flat_adam_hip_skips_nonfinite(bad):
    from ncnet_amd.engine.optim import FlatAdam
    ps = _params("cuda")
    opt = FlatAdam(ps, lr=5e-4)
    opt.zero_grad()
    for p, g in zip(ps, _grads(ps, 0)):
        p.grad.copy_(g)
    opt.mark_loss(torch.tensor(1.0, device="cuda"))
    opt.step()
    before = [p.detach().clone() for p in ps]
    m, v = opt.exp_avg.clone(), opt.exp_avg_sq.clone()
    opt.zero_grad()
    for p, g in zip(ps, _grads(ps, 1)):
        p.grad.copy_(g)
    if bad == "grad":
        ps[2].grad.view(-1)[11] = float("nan")
        opt.mark_loss(torch.tensor(1.0, device="cuda"))
    else:
        opt.mark_loss(torch.tensor(float("inf"), device="cuda"))
    opt.step()
    torch.cuda.synchronize()
    for p, b in zip(ps, before):
        assert torch.equal(p.detach(), b)
    assert torch.equal(opt.exp_avg, m) and torch.equal(opt.exp_avg_sq, v)
    assert opt.steps_taken == 1 and opt.skipped_steps == 1
    assert torch.isfinite(opt.flat_grad[: opt.n]).all()
