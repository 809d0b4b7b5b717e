#!/bin/bash
# InLoc 3200 px bf16 pair latency under launcher knobs (one box, interleaved)
set -u
run() { echo "== $1" >> gpurun_out/inloc_knobs.log; env $1 timeout -k 10 200 python scripts/bench_inloc.py --image-size 3200 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 2>/dev/null | grep '"value"' | cut -c80-125 >> gpurun_out/inloc_knobs.log || exit 1; }
rm -f gpurun_out/inloc_knobs.log
for rep in 1 2; do
  run "NCNET_CORR_NS=3"
  run "NCNET_CORR_NS=4"
  run "NCNET_CONV2D_BIG=1"
  run "NCNET_CONV2D_V3=0"
done
