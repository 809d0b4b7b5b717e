#!/bin/bash
# conv16v4 split tile (20 x 20 planes): oracle / bitwise tests, then the 320 px secondary and the headline
set -u
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_x3.py -k "conv16v4 or wgrad16 or fast1x or x3_fused" > gpurun_out/split_tests.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --only-secondary train --image-size 320 --steps 20 --warmup 5 > gpurun_out/b320.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --only-secondary train --image-size 400 --steps 20 --warmup 5 > gpurun_out/b400.log 2>&1 || exit $?
