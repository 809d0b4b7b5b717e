#!/bin/bash
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/pg"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pg" -o run -- python3 "$ROOT/scripts/prof_pair_graph.py" --image-size ${SIZE:-3200} --pairs 10 --warmup 3 || exit $?
f=$(find "$ROOT/gpurun_out/pg" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/scripts/prof_summary.py" "$f" --marker corr_gemm --warmup 3 --steps 10 --out "$ROOT/gpurun_out/prof_pair_graph_${SIZE:-3200}.md"
rm -rf "$ROOT/gpurun_out/pg"
