#!/bin/bash
# Kernel-trace profile of one bench.py secondary (the timed steps only):
# scripts/prof_secondary.sh TAG "<bench.py args>" WARMUP STEPS -> gpurun_out/sec_TAG.md
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; ARGS=$2; W=${3:-2}; S=${4:-5}
cd /tmp
export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/sec_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sec_$TAG" -o run \
  -- python3 "$ROOT/bench.py" $ARGS --warmup "$W" --steps "$S" || exit $?
f=$(find "$ROOT/gpurun_out/sec_$TAG" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup "$W" --steps "$S" --out "$ROOT/gpurun_out/sec_$TAG.md" || exit $?
rm -rf "$ROOT/gpurun_out/sec_$TAG"
