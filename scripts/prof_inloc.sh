#!/bin/bash
# Kernel-trace profile of the InLoc inference path -> gpurun_out/prof_inloc_<size><tag>.md
#   scripts/prof_inloc.sh [SIZE] [TAG] [extra bench_inloc.py args, e.g. --fp8]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE="${1:-3200}"
TAG="${2:-}"
shift $(( $# > 2 ? 2 : $# ))
cd /tmp
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/prof_inloc$TAG"
rm -rf "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/scripts/bench_inloc.py" --image-size "$SIZE" --pairs ${PAIRS:-3} --warmup 1 "$@" || exit $?
f=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 1 --steps ${PAIRS:-3} --out "$ROOT/gpurun_out/prof_inloc_$SIZE$TAG.md"
