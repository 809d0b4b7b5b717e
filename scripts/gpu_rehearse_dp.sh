#!/bin/bash
# One-GPU box: smoke, a short 1-GPU bench, then the multi-rank bench path
# rehearsed with 2 and 4 ranks on the one card over gloo (RCCL refuses two
# ranks per device; the driver's N=2/4/8 runs use RCCL, one GPU per rank).
set -o pipefail
mkdir -p gpurun_out/dp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/dp/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --inloc 0 > gpurun_out/dp/bench1.log 2>&1 || exit $?
for n in 2 4; do
  NCNET_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 \
    > gpurun_out/dp/bench_gloo$n.log 2>&1 || exit $?
done
tail -n 2 gpurun_out/dp/*.log
