#!/bin/bash
# Round-6 multi-rank rehearsal on ONE MI355X (RCCL refuses two ranks per
# device, so the multi-rank runs use gloo; the driver's 2/4/8-GPU runs use
# RCCL, one GPU per rank):
#  1. RCCL world 1 bench (early NC all-reduce hooks armed: NCNET_FORCE_PG=1);
#  2. bench.py --gpus 2 --batch 32 over gloo (self-launched torchrun);
#  3. train.py under torchrun --nproc-per-node 2 (gloo, synthetic pairs);
#  4. allocator reserved vs peak at the headline batch (scripts/alloc_probe.py).
# Logs -> gpurun_out/r6/dp/
set -o pipefail
OUT=gpurun_out/r6/dp
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
NCNET_FORCE_PG=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 6 --warmup 3 --inloc 0 \
  > $OUT/bench_rccl_world1.log 2>&1 || exit $?
NCNET_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --batch 32 --steps 5 --warmup 2 --inloc 0 \
  > $OUT/bench_gloo2_b32.log 2>&1 || exit $?
NCNET_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 train.py --synthetic 64 --batch_size 8 --num_epochs 1 \
  --image_size 400 --ncons_kernel_sizes 5 5 5 --ncons_channels 16 16 1 --log_interval 2 \
  --result-model-dir /tmp/ncnet_r6_dp --metrics $OUT/train_gloo2_metrics.jsonl > $OUT/train_gloo2.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/alloc_probe.py --batch 256 --steps 4 --warmup 3 > $OUT/alloc_b256.log 2>&1 || exit $?
tail -n 3 $OUT/*.log
