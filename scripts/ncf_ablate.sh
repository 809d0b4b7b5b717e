#!/bin/bash
# Fused InLoc NC kernel: oracle tests, then the 3200 px volume timed under each
# NCNET_NCF_FLAGS ablation (1 tile-major order, 2 / 4 / 8 skip layer 1 / layer 2 / gather)
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "nc_fused" > gpurun_out/ncf_tests.log 2>&1 || exit $?
for f in ${NCF_FLAG_LIST:-0 16 32 48 1 2 4 8 14 0}; do
  echo "flags=$f" >> gpurun_out/ncf_ablate.log
  NCNET_NCF_FLAGS=$f timeout -k 10 120 python scripts/nc_fused_bench.py --reps 10 >> gpurun_out/ncf_ablate.log 2>&1 || exit $?
done
