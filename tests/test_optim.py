"""FlatAdam (engine/optim.py): torch.optim.Adam numerics, Adam-layout state
dicts, and the exact NaN/Inf step skip -- single process and 2-rank gloo DP
(a non-finite loss on ONE rank makes EVERY rank skip the step)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ncnet_amd.engine.optim import FlatAdam
from ncnet_amd.parallel.dist import DistContext, GradBucket


def _params(seed=0, dev="cpu"):
    g = torch.Generator().manual_seed(seed)
    shapes = [(5, 16, 1, 5, 5, 5), (16,), (3, 7), (1,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]


def _grads(params, step, scale=1.0):
    g = torch.Generator().manual_seed(1000 + step)
    return [scale * torch.randn(p.shape, generator=g).to(p.device) for p in params]


@pytest.mark.parametrize("wd", [0, 1e-2])
def test_flat_adam_matches_torch_adam(wd):
    pa, pb = _params(), _params()
    ta = torch.optim.Adam(pa, lr=5e-4, weight_decay=wd)
    fb = FlatAdam(pb, lr=5e-4, weight_decay=wd)
    for step in range(6):
        ta.zero_grad()
        fb.zero_grad()
        for p, q, g in zip(pa, pb, _grads(pa, step)):
            p.grad = g.clone()
            q.grad.copy_(g)          # .grad is a view into the flat buffer
        ta.step()
        fb.step()
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-6, atol=1e-7)
    assert fb.steps_taken == 6 and fb.skipped_steps == 0


def test_flat_adam_grads_are_bucket_views():
    ps = _params()
    opt = FlatAdam(ps, lr=1e-3)
    opt.zero_grad(set_to_none=True)    # views survive set_to_none
    loss = sum((p * p).sum() for p in ps)
    loss.backward()
    flat = torch.cat([(2 * p.detach()).reshape(-1) for p in ps])
    torch.testing.assert_close(opt.flat_grad[: opt.n], flat)
    for p in ps:
        assert p.grad.untyped_storage().data_ptr() == opt.flat_grad.untyped_storage().data_ptr()


def test_state_dict_interchanges_with_torch_adam():
    pa, pb, pc = _params(), _params(), _params()
    fa = FlatAdam(pa, lr=5e-4)
    for step in range(3):
        fa.zero_grad()
        for p, g in zip(pa, _grads(pa, step)):
            p.grad.copy_(g)
        fa.step()
    sd = fa.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"} and float(sd["state"][0]["step"]) == 3.0
    # torch Adam continues from FlatAdam's state ...
    with torch.no_grad():
        for p, q in zip(pb, pa):
            p.copy_(q)
    ta = torch.optim.Adam(pb, lr=5e-4)
    ta.load_state_dict(sd)
    # ... and FlatAdam continues from torch Adam's state
    with torch.no_grad():
        for p, q in zip(pc, pa):
            p.copy_(q)
    fc = FlatAdam(pc, lr=5e-4)
    fc.load_state_dict(ta.state_dict())
    for step in range(3, 5):
        ta.zero_grad()
        fc.zero_grad()
        for p, q, g in zip(pb, pc, _grads(pb, step)):
            p.grad = g.clone()
            q.grad.copy_(g)
        ta.step()
        fc.step()
    for p, q in zip(pb, pc):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("where", ["grad_nan", "grad_inf", "loss_nan", "loss_inf"])
def test_nonfinite_step_is_skipped_exactly(where):
    ps = _params()
    opt = FlatAdam(ps, lr=5e-4)
    for step in range(2):
        opt.zero_grad()
        for p, g in zip(ps, _grads(ps, step)):
            p.grad.copy_(g)
        opt.mark_loss(torch.tensor(1.0))
        opt.step()
    before = [p.detach().clone() for p in ps]
    m, v = opt.exp_avg.clone(), opt.exp_avg_sq.clone()
    opt.zero_grad()
    for p, g in zip(ps, _grads(ps, 7)):
        p.grad.copy_(g)
    bad = float("nan") if where.endswith("nan") else float("inf")
    if where.startswith("grad"):
        ps[0].grad.view(-1)[3] = bad
        opt.mark_loss(torch.tensor(1.0))
    else:
        opt.mark_loss(torch.tensor(bad))
    opt.step()
    for p, b in zip(ps, before):
        assert torch.equal(p.detach(), b)
    assert torch.equal(opt.exp_avg, m) and torch.equal(opt.exp_avg_sq, v)
    assert opt.steps_taken == 2 and opt.skipped_steps == 1
    assert torch.isfinite(opt.flat_grad[: opt.n]).all()   # the skipped step's gradients are zeroed
    # training continues normally afterwards
    opt.zero_grad()
    for p, g in zip(ps, _grads(ps, 8)):
        p.grad.copy_(g)
    opt.mark_loss(torch.tensor(1.0))
    opt.step()
    assert opt.steps_taken == 3 and not torch.equal(ps[0].detach(), before[0])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from ncnet_amd.parallel.dist import destroy, init_distributed
    ctx = init_distributed(device="cpu")
    ps = _params()
    opt = FlatAdam(ps, lr=5e-4)
    bucket = GradBucket(ps, ctx, opt)
    assert bucket.inplace and opt.grad_scale == 1.0 / world
    hist = []
    for step in range(3):
        opt.zero_grad()
        for p, g in zip(ps, _grads(ps, 10 * step + rank)):
            p.grad.copy_(g)
        loss = torch.tensor(float("nan") if (step == 1 and rank == 1) else 1.0)
        opt.mark_loss(loss)
        bucket.allreduce()
        opt.step()
        hist.append([p.detach().clone() for p in ps])
    torch.save({"hist": hist, "steps": opt.steps_taken, "skipped": opt.skipped_steps},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy(ctx)


def test_dp_nonfinite_on_one_rank_skips_on_all(tmp_path):
    world = 2
    mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in res:
        assert r["steps"] == 2 and r["skipped"] == 1
        for a, b in zip(r["hist"][0], r["hist"][1]):
            assert torch.equal(a, b)           # step 1 skipped on BOTH ranks
    for a, b in zip(res[0]["hist"][2], res[1]["hist"][2]):
        assert torch.equal(a, b)               # ranks stay in lock-step
    # the averaged update equals a single-process Adam on the mean gradient
    ps = _params()
    ta = torch.optim.Adam(ps, lr=5e-4)
    for step in (0, 2):
        ta.zero_grad()
        gs = [_grads(ps, 10 * step + r) for r in range(world)]
        for i, p in enumerate(ps):
            p.grad = sum(g[i] for g in gs) / world
        ta.step()
    for p, q in zip(ps, res[0]["hist"][2]):
        torch.testing.assert_close(q, p.detach(), rtol=1e-6, atol=1e-7)


def test_bucket_inplace_world1_without_pg_is_noop():
    ps = _params()
    opt = FlatAdam(ps, lr=1e-3)
    b = GradBucket(ps, DistContext(), opt)
    assert b.inplace and opt.grad_scale == 1.0
    b.allreduce()


def test_rebound_parameter_raises():
    """A module moved after make_adam detaches its parameters from the flat
    buffers; step() must say so instead of updating storage nobody reads."""
    m = torch.nn.Linear(4, 3)
    opt = FlatAdam(list(m.parameters()), lr=1e-3)
    opt.zero_grad()
    m(torch.randn(2, 4)).sum().backward()
    opt.step()                                   # bound: fine
    m.double()                                   # module._apply: new storage
    with pytest.raises(RuntimeError, match="no longer a view"):
        opt.step()


def test_guard_off_applies_nonfinite_step():
    """Trainer(nan_guard=False) -> FlatAdam.guard False: no skip."""
    p = _params()
    opt = FlatAdam(p, lr=1e-3)
    opt.guard = False
    opt.zero_grad()
    for q in p:
        q.grad.fill_(1.0)
    p[0].grad.view(-1)[0] = float("nan")
    opt.step()
    assert opt.skipped_steps == 0 and opt.steps_taken == 1
    assert torch.isnan(p[0].detach().view(-1)[0])
