#!/bin/bash
# Kernel-trace profile of the InLoc inference path (eval_inloc.py's schedule:
# 10 panos per query, pair HIP graph) -> gpurun_out/prof_inloc_<size><tag>.md,
# steady state: the first query is warm-up, the summary covers the next ones.
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
Q=${QUERIES:-2}
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/scripts/bench_inloc.py" --image-size "$SIZE" --panos-per-query 10 --pairs $((10 * Q)) \
  --warmup 10 "$@" > "$OUT.log" 2>&1 || exit $?
f=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --marker l2norm_rows_kernel --warmup 1 --steps $Q \
  --out "$ROOT/gpurun_out/prof_inloc_$SIZE$TAG.md" > /dev/null
rm -rf "$OUT"
