#!/bin/bash
# Interleaved same-box A/B of bench.py (box-to-box spread ~5 % exceeds most
# single changes): scripts/gpu_ab2.sh TAG ROUNDS "ENV=V ..." "ENV=V ..." [...]
# runs config 1, 2, ... then again, ROUNDS times; one JSON value per line.
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/$TAG
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inloc 0 > gpurun_out/$TAG/ab_${i}_$r.log 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' gpurun_out/$TAG/ab_${i}_$r.log | head -1)
    echo "[$cfg] round $r: $v"
    i=$((i+1))
  done
done
