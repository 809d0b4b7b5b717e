#!/bin/bash
# fused-NC tests + kernel timing + InLoc 3200 / 1600 bf16 pair latency
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "nc_fused or fused_symmetric" > gpurun_out/ncf_tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/nc_fused_bench.py --reps 20 --sweep "${NCF_SWEEP:-}" > gpurun_out/ncf_bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_inloc.py --image-size 3200 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 > gpurun_out/inloc3200.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_inloc.py --image-size 1600 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 > gpurun_out/inloc1600.log 2>&1 || exit $?
