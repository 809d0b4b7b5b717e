"""Multi-rank data-parallel training rehearsed on ONE MI355X (RCCL refuses two
ranks per device, so the collectives run over gloo; the driver's 2/4/8-GPU
runs use RCCL, one GPU per rank).  Two ranks train the headline model
(ResNet-101 + NC 5,5,5 / 16,16,1, 400 px: the compile-time fast kernels, the
side-stream weight gradients of ops/neigh_consensus.py and the trunk
prefetch) through the real Trainer -- flat gradient bucket all-reduce, FlatAdam
with the 1/world average folded in -- and must end bit-identical to each other
and equal to ONE process doing FlatAdam on the mean of the two shards'
gradients.  Also records each rank's allocator
reserved vs peak (the round-5 side-stream lifetime change must keep the
reserved pool near the peak)."""
import json
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed, b=2, size=400):
    g = torch.Generator().manual_seed(seed)
    return {"source_image": torch.randn(b, 3, size, size, generator=g),
            "target_image": torch.randn(b, 3, size, size, generator=g)}


def _worker(rank, world, port, out_dir, steps):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), NCNET_DIST_BACKEND="gloo")
    import dataclasses
    from ncnet_amd import config
    config.set_runtime(dataclasses.replace(config.RuntimeConfig.from_env(), trunk_conv="native"))
    # the MIOpen stem with a fixed solver in every process (as the reference below)
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import broadcast_module, destroy, init_distributed
    ctx = init_distributed()
    torch.manual_seed(300 + rank)                 # different init on purpose: broadcast must fix it
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").to(ctx.device)
    m.train()
    params = [p for p in m.parameters() if p.requires_grad]
    broadcast_module(m, ctx)
    init = [p.detach().clone().cpu() for p in params]
    tr = Trainer(m, make_adam(params, 5e-4), ctx)
    torch.cuda.reset_peak_memory_stats()
    for step in range(steps):
        tr.train_step(tr.to_device(_batch(1000 * step + rank)))
    torch.cuda.synchronize()
    st = torch.cuda.memory_stats()
    torch.save({"init": init, "params": [p.detach().clone().cpu() for p in params],
                "mem": {"reserved_peak_gb": st["reserved_bytes.all.peak"] / 2 ** 30,
                        "allocated_peak_gb": st["allocated_bytes.all.peak"] / 2 ** 30,
                        "alloc_retries": st["num_alloc_retries"]}},
               os.path.join(out_dir, f"r{rank}.pt"))
    destroy(ctx)


def _reference_worker(_, world, out_dir, steps):
    """ONE process doing FlatAdam on the summed shard gradients (g0 + g1, the
    in-place summed bucket, 1/world folded into the step as GradBucket sets
    it) -- in a fresh process like the ranks, so no state left by earlier
    tests in the pytest process (MIOpen solver caches, runtime knobs) enters
    the comparison."""
    import dataclasses
    from ncnet_amd import config
    config.set_runtime(dataclasses.replace(config.RuntimeConfig.from_env(), trunk_conv="native"))
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    from ncnet_amd.engine.trainer import make_adam, weak_loss
    from ncnet_amd.models import ImMatchNet
    init = torch.load(os.path.join(out_dir, "r0.pt"), weights_only=True)["init"]
    torch.manual_seed(300)
    m = ImMatchNet(ncons_kernel_sizes=[5, 5, 5], ncons_channels=[16, 16, 1], dtype="bf16").cuda()
    m.train()
    params = [p for p in m.parameters() if p.requires_grad]
    with torch.no_grad():
        for p, v in zip(params, init):
            p.copy_(v.cuda())
    opt = make_adam(params, 5e-4)
    opt.grad_scale = 1.0 / world
    for step in range(steps):
        opt.zero_grad()
        for r in range(world):             # shard gradients accumulate into the flat buffer: g0 + g1
            b = {k: v.cuda() for k, v in _batch(1000 * step + r).items()}
            weak_loss(m, b).backward()
        opt.step()
    torch.cuda.synchronize()
    torch.save([p.detach().clone().cpu() for p in params], os.path.join(out_dir, "ref.pt"))


def test_dp2_gloo_on_one_gpu_equals_single_process(tmp_path):
    world, steps = 2, 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), steps), nprocs=world, join=True)
    res = [torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True) for r in range(world)]
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b)
    mp.spawn(_reference_worker, args=(world, str(tmp_path), steps), nprocs=1, join=True)
    ref = torch.load(str(tmp_path / "ref.pt"), weights_only=True)
    # same kernels and shapes per shard; the all-reduce sums two fp32 values
    # (exact either way round), FlatAdam scales by 1/world in-kernel
    for a, p in zip(res[0]["params"], ref):
        assert torch.allclose(a, p, rtol=1e-5, atol=1e-6), float((a - p).abs().max())
    mem = [r["mem"] for r in res]
    out = os.path.join(ROOT, "gpurun_out", "dp_rehearsal_mem.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(mem, f)
    for mm in mem:
        assert mm["alloc_retries"] == 0, mm
        assert mm["reserved_peak_gb"] <= 1.5 * mm["allocated_peak_gb"] + 2.0, mm
