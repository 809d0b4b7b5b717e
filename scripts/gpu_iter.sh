#!/bin/bash
# One GPU iteration: a pytest subset, a kbench subset, a short 1-GPU bench.
# usage: scripts/gpu_iter.sh "<pytest -k expr or empty>" "<kbench --only list or empty>" [bench 0|1] [tag]
set -o pipefail
TAG="${4:-iter}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$1" \
    > $OUT/pytest.log 2>&1
  rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$2" ]; then
  timeout -k 10 300 python -u scripts/kbench.py --reps 10 --only "$2" > $OUT/kbench.log 2>&1
  rc=$?; cat $OUT/kbench.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
fi
if [ "${3:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inloc 0 > $OUT/bench.log 2>&1
  rc=$?; tail -n 1 $OUT/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
exit 0
