#!/bin/bash
# Per-GPU batch sweep of the headline step (BASELINE config 3: DP batch sized
# for 288 GB HBM) -> gpurun_out/$TAG/b<N>.log, one JSON record each (hbm_peak_gb)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r5/batch}
mkdir -p "$ROOT/gpurun_out/$TAG"
for B in ${BATCHES:-16 32 64 128}; do
  timeout -k 10 600 python3 "$ROOT/bench.py" --batch "$B" --steps ${STEPS:-10} --warmup 3 --inloc 0 \
    > "$ROOT/gpurun_out/$TAG/b$B.log" 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"hbm_peak_gb": [0-9.]*\|"ms_per_step": [0-9.]*' "$ROOT/gpurun_out/$TAG/b$B.log" | tr '\n' ' '
  echo " batch $B"
done
