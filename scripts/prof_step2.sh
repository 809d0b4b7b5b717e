#!/bin/bash
# Kernel-trace profiles of bench.py's timed steps, pipelined (default) and
# serial (NCNET_TRUNK_PREFETCH=0 NCNET_BWD_OVERLAP=0: clean per-kernel times)
# -> gpurun_out/step_{pipelined,serial}.md
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp
export TMPDIR=/tmp
for mode in pipelined serial; do
  rm -rf "$ROOT/gpurun_out/prof_$mode"
  if [ "$mode" = serial ]; then export NCNET_TRUNK_PREFETCH=0 NCNET_BWD_OVERLAP=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/prof_$mode" -o run \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --inloc 0 || exit $?
  f=$(find "$ROOT/gpurun_out/prof_$mode" -name "*kernel_trace.csv" | head -1)
  python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 3 --steps 5 --out "$ROOT/gpurun_out/step_$mode.md" || exit $?
  rm -rf "$ROOT/gpurun_out/prof_$mode"
done
