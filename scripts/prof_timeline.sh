#!/bin/bash
# Kernel trace of bench.py (pipelined step) -> gpurun_out/$TAG/timeline_step*.md
# usage: [BENCH_ARGS="--batch 512"] scripts/prof_timeline.sh TAG [extra env assignments...]
set -u
TAG=${1:-timeline}; shift || true
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/$TAG"
rm -rf "$OUT/trace"; mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --steps 6 --warmup 3 --inloc 0 ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || exit $?
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_timeline.py" "$f" --step 5 --marker corr_gemm --out "$OUT/timeline_step5.md" > /dev/null || exit $?
python3 "$ROOT/scripts/prof_timeline.py" "$f" --step 6 --marker corr_gemm --out "$OUT/timeline_step6.md" > /dev/null || exit $?
python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 3 --steps 6 --out "$OUT/summary.md" > /dev/null
rm -rf "$OUT/trace"
