#!/bin/bash
# Kernel-trace A/B of bench.py's timed steps: for each "NAME:ENV=V,ENV2=V2"
# argument, one rocprofv3 --kernel-trace run with that environment, summarised
# to gpurun_out/<tag>/step_<NAME>.md (scripts/prof_summary.py).
#   scripts/prof_ab.sh <tag> <name:env,...> [<name:env,...> ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  (
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [ -n "$e" ] && export "$e"; done
    rm -rf "$OUT/prof_$name"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$name" -o run \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --inloc 0 > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || exit $?
    f=$(find "$OUT/prof_$name" -name "*kernel_trace.csv" | head -1)
    python3 "$ROOT/scripts/prof_summary.py" "$f" --warmup 3 --steps 5 --out "$OUT/step_$name.md" || exit $?
    rm -rf "$OUT/prof_$name"
  ) || exit $?
  echo "$name done"
done
