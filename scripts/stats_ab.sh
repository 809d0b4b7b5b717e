#!/bin/bash
set -u
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_property.py tests/test_gpu_cli.py -k "stats or mutual or loss or match or inloc" > gpurun_out/stats_tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_inloc.py --image-size 3200 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 > gpurun_out/inloc3200.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_inloc.py --image-size 1600 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 > gpurun_out/inloc1600.log 2>&1 || exit $?
