#!/bin/bash
# Kernel-trace profile of bench.py timed steps -> gpurun_out/prof_summary.md
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp
export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/prof"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/prof" -o run \
  -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 || exit $?
f=$(find "$ROOT/gpurun_out/prof" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 3 --steps 5 --out "$ROOT/gpurun_out/prof_summary.md"
