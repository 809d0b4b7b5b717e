#!/bin/bash
# A/B of bench.py under environment settings: scripts/gpu_ab.sh tag "ENV=V ..." ["ENV=V ..."] ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for cfg in "$@"; do
  for rep in 1 2; do
    env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inloc 0 > gpurun_out/$TAG/ab_${i}_$rep.log 2>&1 || exit $?
    echo "[$cfg] rep $rep: $(tail -n 1 gpurun_out/$TAG/ab_${i}_$rep.log | cut -c1-160)"
  done
  i=$((i+1))
done
