"""Data-parallel correctness over gloo on CPU (world sizes 2 .. 8).

DP semantics: each rank computes the weak loss on
its own shard with its own negative roll; the averaged gradient must equal the
mean of the per-shard gradients computed in a single process."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    return {"source_image": torch.randn(2, 3, 64, 64, generator=g), "target_image": torch.randn(2, 3, 64, 64, generator=g)}


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1 if world > 4 else 2)
    from ncnet_amd.engine.trainer import weak_loss
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import GradBucket, broadcast_module, destroy, init_distributed, shard_indices
    ctx = init_distributed(device="cpu")
    assert ctx.backend == "gloo" and ctx.world_size == world
    torch.manual_seed(100 + rank)  # different init on purpose: broadcast must fix it
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    params = [p for p in m.parameters() if p.requires_grad]
    broadcast_module(m, ctx)
    loss = weak_loss(m, _batch(rank))
    loss.backward()
    GradBucket(params, ctx).allreduce()
    torch.save({"state": m.state_dict(), "params": [p.detach() for p in params], "grads": [p.grad for p in params],
                "shard": shard_indices(10, ctx, epoch=0)}, os.path.join(out_dir, f"r{rank}.pt"))
    destroy(ctx)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gradients_equal_mean_of_shards(tmp_path, world):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in range(1, world):
        for a, b in zip(res[0]["params"], res[r]["params"]):
            assert torch.equal(a, b)  # broadcast from rank 0
        for a, b in zip(res[0]["grads"], res[r]["grads"]):
            assert torch.allclose(a, b)
    # single-process reference with rank 0's parameters, at the workers' thread
    # count: the same kernels in the same order per shard (the weak loss at random
    # init sits in near-ties of its argmaxes; another summation order can flip one)
    from ncnet_amd.engine.trainer import weak_loss
    from ncnet_amd.models import ImMatchNet
    nthr = torch.get_num_threads()
    torch.set_num_threads(1 if world > 4 else 2)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    m.load_state_dict(res[0]["state"])
    params = [p for p in m.parameters() if p.requires_grad]
    acc = [torch.zeros_like(p) for p in params]
    for r in range(world):
        m.zero_grad()
        weak_loss(m, _batch(r)).backward()
        for a, p in zip(acc, params):
            a += p.grad / world
    torch.set_num_threads(nthr)
    for a, g in zip(acc, res[0]["grads"]):
        assert torch.allclose(a, g, rtol=1e-4, atol=1e-8), (float((a - g).abs().max()), float(a.abs().max()))
    # disjoint, equal-size shards (drop_last: 10 // world pairs per rank, as DistributedSampler)
    shards = [set(r["shard"]) for r in res]
    assert sum(len(x) for x in shards) == len(set().union(*shards)) == world * (10 // world)
    assert all(len(r["shard"]) == 10 // world for r in res)


def test_bench_torchrun_two_ranks_cpu(tmp_path):
    """The driver's multi-GPU launch line, on CPU/gloo at a toy size: two ranks,
    one JSON line from rank 0 with whole-job throughput and dp2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2", NCNET_FORCE_TORCH="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29731", os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--batch", "2", "--image-size", "64"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 4
    assert rec["value"] > 0 and rec["steps"] == 1 and rec["warmup"] == 1


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launch_cpu(tmp_path, world):
    """Plain ``python bench.py --gpus N`` (no launcher env): bench.py starts
    torch.distributed.run itself as a child process and relays rank 0's record;
    the record must say N ranks with a real process group and whole-job
    throughput (the driver's 8-GPU scaling run, rehearsed on gloo)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID")}
    env.update(OMP_NUM_THREADS="1" if world > 4 else "2", NCNET_FORCE_TORCH="1")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--steps", "1", "--warmup", "1",
           "--batch", "2", "--image-size", "64"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world and rec["config"]["parallelism"] == f"dp{world}"
    assert rec["config"]["global_batch"] == 2 * world
    assert rec["config"]["comm"]["process_group"] is True and rec["config"]["comm"]["world_size"] == world
    assert rec["config"]["launcher"] == "self-launched torchrun"


def test_bench_world_mismatch_fails(tmp_path):
    """--gpus 1 inside a 2-rank launch must fail instead of timing a wrong job."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2", NCNET_FORCE_TORCH="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29735", os.path.join(root, "bench.py"), "--gpus", "1", "--steps", "1",
           "--warmup", "0", "--batch", "1", "--image-size", "64"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


@pytest.mark.parametrize("world", [2, 8])
def test_train_torchrun_cpu(tmp_path, world):
    """train.py under torchrun with N gloo ranks: the Trainer's one-batch
    lookahead loop (TrunkPrefetcher hand-off), sharded sampler, gradient
    bucket and rank-0 checkpointing run end to end."""
    import glob
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1" if world > 4 else "2", NCNET_FORCE_TORCH="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "train.py"),
           "--synthetic", str(4 * world),
           "--batch_size", "2", "--image_size", "64", "--ncons_kernel_sizes", "3", "3", "--ncons_channels", "16", "1",
           "--num_epochs", "1", "--result-model-dir", "models"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Train Epoch: 1" in out.stdout and "Test set: Average loss" in out.stdout
    assert glob.glob(str(tmp_path / "models" / "*_checkpoint_adam.pth.tar"))


def _vp_worker(rank, world, port, out_dir, k_size, ks):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import broadcast_module, destroy, init_distributed
    from ncnet_amd.parallel.volume_parallel import VolumeParallelMatcher
    ctx = init_distributed(device="cpu")
    torch.manual_seed(7)
    m = ImMatchNet(ncons_kernel_sizes=ks, ncons_channels=[16] * (len(ks) - 1) + [1], use_cuda=False,
                   relocalization_k_size=k_size).eval()
    broadcast_module(m, ctx)
    g = torch.Generator().manual_seed(3)
    batch = {"source_image": torch.randn(1, 3, 256, 192, generator=g),
             "target_image": torch.randn(1, 3, 192, 256, generator=g)}
    out = VolumeParallelMatcher(m, ctx).forward(batch)
    if rank == 0:
        torch.save({"state": m.state_dict(), "out": out, "batch": batch}, os.path.join(out_dir, "vp.pt"))
    destroy(ctx)


@pytest.mark.parametrize("world,k_size,ks", [(2, 2, [3, 3]), (3, 1, [3, 3]), (2, 2, [5, 3])])
def test_volume_parallel_matches_single_process(tmp_path, world, k_size, ks):
    """A-row-sharded correlation / MutualMatching / NeighConsensus (one halo
    exchange) / MutualMatching over gloo == the single-process model."""
    port = _free_port()
    mp.spawn(_vp_worker, args=(world, port, str(tmp_path), k_size, ks), nprocs=world, join=True)
    res = torch.load(str(tmp_path / "vp.pt"), weights_only=True)
    from ncnet_amd.models import ImMatchNet
    m = ImMatchNet(ncons_kernel_sizes=ks, ncons_channels=[16] * (len(ks) - 1) + [1], use_cuda=False,
                   relocalization_k_size=k_size).eval()
    m.load_state_dict(res["state"])
    with torch.inference_mode():
        ref = m(res["batch"])
    if k_size > 1:
        corr, delta = res["out"]
        rc, rd = ref
        assert corr.shape == rc.shape
        assert torch.allclose(corr, rc, rtol=1e-4, atol=1e-6)
        for a, b in zip(delta, rd):
            assert torch.equal(a.long(), b.long())
    else:
        assert res["out"].shape == ref.shape
        assert torch.allclose(res["out"], ref, rtol=1e-4, atol=1e-6)


def _hang_worker(rank, world, port, out_dir):
    """Rank 1 never joins the all-reduce (a hung or dead peer); rank 0 must get
    an error from the process-group timeout instead of blocking forever."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import time
    from ncnet_amd.parallel.dist import init_distributed
    ctx = init_distributed(device="cpu", timeout_s=5)
    if rank == 1:
        time.sleep(30)           # stays alive but silent past the timeout
        return
    import torch.distributed as dist
    t0 = time.time()
    err = ""
    try:
        dist.all_reduce(torch.ones(4))
    except Exception as e:        # gloo: RuntimeError "... Timed out ..."
        err = repr(e)
    with open(os.path.join(out_dir, "hang.txt"), "w") as f:
        f.write(f"{time.time() - t0:.1f}\n{err}")
    os._exit(0)                   # do not wait for the silent peer in destroy()


def test_rank_failure_detected_by_pg_timeout(tmp_path):
    """SURVEY 5.3 failure detection: with NCNET_PG_TIMEOUT_S-style timeouts a
    collective that a peer never joins raises on the surviving rank within the
    timeout (parallel/dist.py init_distributed)."""
    port = _free_port()
    ctx = mp.spawn(_hang_worker, args=(2, port, str(tmp_path)), nprocs=2, join=False)
    ctx.processes[0].join(120)
    assert not ctx.processes[0].is_alive(), "rank 0 blocked past the process-group timeout"
    for p in ctx.processes:
        if p.is_alive():
            p.terminate()
            p.join(10)
    elapsed, err = (tmp_path / "hang.txt").read_text().split("\n", 1)
    assert err, "the all-reduce with a silent peer did not raise"
    assert float(elapsed) < 60


def _overlap_worker(rank, world, port, out_dir, early):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import broadcast_module, destroy, init_distributed
    ctx = init_distributed(device="cpu")
    torch.manual_seed(7)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    for p in m.FeatureExtraction.model[-1][-1].parameters():      # --fe_finetune_params 1
        p.requires_grad = True
    params = [p for p in m.parameters() if p.requires_grad]
    broadcast_module(m, ctx)
    tr = Trainer(m, make_adam(params, 5e-4), ctx)
    if not early:
        tr.bucket._early_seg = None                                 # the serial single-bucket path
    for step in range(2):
        tr.train_step(_batch(10 * step + rank))
    launches = getattr(tr.bucket, "early_launches", 0) if early else 0
    snap = [p.detach().clone() for p in params]
    stale = 0
    if early:
        # a second trainer on the same parameters (a restart in-process): the
        # first bucket's hooks must stay silent (disarmed after its finish)
        old = tr.bucket
        tr2 = Trainer(m, make_adam(params, 5e-4), ctx)
        tr2.train_step(_batch(99 + rank))
        stale = old.early_launches - launches
        assert tr2.bucket.early_launches == 1
        old.close()
        tr2.bucket.close()
        assert not old._hooks and not tr2.bucket._hooks
    torch.save({"params": snap, "early_launches": launches, "stale": stale},
               os.path.join(out_dir, f"{'e' if early else 's'}{rank}.pt"))
    destroy(ctx)


def test_early_nc_allreduce_matches_serial(tmp_path):
    """GradBucket early segment (NC gradients all-reduced from a post-accumulate
    hook while autograd continues into the trainable backbone) gives the same
    parameters, bit for bit, as one bucket all-reduced after backward."""
    world = 2
    for early in (True, False):
        mp.spawn(_overlap_worker, args=(world, _free_port(), str(tmp_path), early), nprocs=world, join=True)
    for r in range(world):
        e = torch.load(str(tmp_path / f"e{r}.pt"), weights_only=True)
        s = torch.load(str(tmp_path / f"s{r}.pt"), weights_only=True)
        assert e["early_launches"] == 2                            # one per step, from the hook
        assert e["stale"] == 0                                     # the replaced bucket launched nothing
        for a, b in zip(e["params"], s["params"]):
            assert torch.equal(a, b)


def _train_worker(rank, world, port, out_dir, steps):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from ncnet_amd.engine.trainer import Trainer, make_adam
    from ncnet_amd.models import ImMatchNet
    from ncnet_amd.parallel.dist import broadcast_module, destroy, init_distributed
    ctx = init_distributed(device="cpu")
    torch.manual_seed(200 + rank)      # different init on purpose: broadcast must fix it
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    params = [p for p in m.parameters() if p.requires_grad]
    broadcast_module(m, ctx)
    init = [p.detach().clone() for p in params]
    tr = Trainer(m, make_adam(params, 5e-3), ctx)
    for step in range(steps):
        tr.train_step(_batch(1000 * step + rank))
    torch.save({"init": init, "params": [p.detach().clone() for p in params]}, os.path.join(out_dir, f"t{rank}.pt"))
    destroy(ctx)


def test_dp_training_world8_equals_single_process(tmp_path):
    """Eight gloo ranks train two steps through the real Trainer (flat gradient
    bucket all-reduce, FlatAdam with the 1/world average folded in): every rank
    ends with the same parameters, equal to one process doing Adam on the mean
    of the eight shard gradients."""
    world, steps = 8, 2
    mp.spawn(_train_worker, args=(world, _free_port(), str(tmp_path), steps), nprocs=world, join=True)
    res = [torch.load(str(tmp_path / f"t{r}.pt"), weights_only=True) for r in range(world)]
    for r in range(1, world):
        for a, b in zip(res[0]["params"], res[r]["params"]):
            assert torch.equal(a, b)
    from ncnet_amd.engine.trainer import weak_loss
    from ncnet_amd.models import ImMatchNet
    nthr = torch.get_num_threads()
    torch.set_num_threads(1)                   # the workers' kernels and summation order
    torch.manual_seed(200)
    m = ImMatchNet(ncons_kernel_sizes=[3, 3], ncons_channels=[16, 1], use_cuda=False)
    params = [p for p in m.parameters() if p.requires_grad]
    with torch.no_grad():
        for p, v in zip(params, res[0]["init"]):
            p.copy_(v)
    opt = torch.optim.Adam(params, lr=5e-3)
    for step in range(steps):
        acc = [torch.zeros_like(p) for p in params]
        for r in range(world):
            m.zero_grad()
            weak_loss(m, _batch(1000 * step + r)).backward()
            for a, p in zip(acc, params):
                a += p.grad / world
        for p, a in zip(params, acc):
            p.grad = a
        opt.step()
    torch.set_num_threads(nthr)
    # Adam at random init divides ~1e-8 gradients by sqrt(v) ~ eps: the all-reduce's
    # summation order and the in-kernel 1/world scale move an update by ~0.1 % of
    # its lr-sized step (5e-3), far below one step
    for a, p in zip(res[0]["params"], params):
        assert torch.allclose(a, p.detach(), rtol=1e-4, atol=2e-5), float((a - p).abs().max())
