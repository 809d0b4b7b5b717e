#!/bin/bash
# Kernel-trace profile of the InLoc inference path -> gpurun_out/prof_inloc_<size>.md
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE="${1:-3200}"
cd /tmp
export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/prof_inloc"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/prof_inloc" -o run \
  -- python3 "$ROOT/scripts/bench_inloc.py" --image-size "$SIZE" --pairs 3 --warmup 1 || exit $?
f=$(find "$ROOT/gpurun_out/prof_inloc" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 1 --steps 3 --out "$ROOT/gpurun_out/prof_inloc_$SIZE.md"
