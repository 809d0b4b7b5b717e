#!/bin/bash
# Per-kernel stats of the frozen trunk alone (scripts/time_trunk.py) at the
# InLoc (11 x 2400x3200) and training (32 x 400x400) shapes -> gpurun_out/trunk_*_stats.csv
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp
export TMPDIR=/tmp
for cfg in "3200:11:2400 3200" "400:32:400 400"; do
  tag="${cfg%%:*}"; rest="${cfg#*:}"; b="${rest%%:*}"; hw="${rest#*:}"
  rm -rf "$ROOT/gpurun_out/trunk_$tag"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/trunk_$tag" -o run \
    -- python3 "$ROOT/scripts/time_trunk.py" --batch "$b" --hw $hw --iters 10 || exit $?
  f=$(find "$ROOT/gpurun_out/trunk_$tag" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$ROOT/gpurun_out/trunk_${tag}_stats.csv"
  rm -rf "$ROOT/gpurun_out/trunk_$tag"
done
