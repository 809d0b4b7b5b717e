#!/bin/bash
# Kernel-trace profile of the frozen trunk alone -> gpurun_out/prof_trunk_<tag>.md
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
cd /tmp
export TMPDIR=/tmp NCNET_TRUNK_GRAPH=0
rm -rf "$ROOT/gpurun_out/prof_trunk"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/prof_trunk" -o run \
  -- python3 "$ROOT/scripts/time_trunk.py" "$@" || exit $?
f=$(find "$ROOT/gpurun_out/prof_trunk" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 3 --steps 10 --marker bias_act_kernel --out "$ROOT/gpurun_out/prof_trunk_$TAG.md"
