#!/bin/bash
# Kernel stats of the headline bench under torchrun --nproc-per-node 1 (RCCL
# process group, world 1) vs plain python (no process group): where the
# process-group step's extra time goes -> gpurun_out/tr1_{pg,nopg}_stats.csv
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp
export TMPDIR=/tmp
rm -rf "$ROOT/gpurun_out/tr1_pg" "$ROOT/gpurun_out/tr1_nopg"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/tr1_nopg" -o run \
  -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --inloc 0 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/tr1_pg" -o run \
  -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 \
  "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --inloc 0 || exit $?
for t in pg nopg; do
  f=$(find "$ROOT/gpurun_out/tr1_$t" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$ROOT/gpurun_out/tr1_${t}_stats.csv"
  k=$(find "$ROOT/gpurun_out/tr1_$t" -name "*kernel_trace.csv" | head -1)
  python3 "$ROOT/scripts/prof_summary.py" "$k" --warmup 5 --steps 20 --out "$ROOT/gpurun_out/tr1_${t}_summary.md" || true
  rm -rf "$ROOT/gpurun_out/tr1_$t"
done
