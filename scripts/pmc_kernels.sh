#!/bin/bash
# PMC counter passes over the NC kernel microbench (kernel-trace-free, one
# counter group per rocprofv3 run). Writes gpurun_out/pmc_<pass>/ CSVs.
# usage: scripts/pmc_kernels.sh "<kbench --only list>"
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ONLY="$1"
cd /tmp
export TMPDIR=/tmp PYTHONPATH="$ROOT"
rocprofv3 -L > "$ROOT/gpurun_out/pmc_list.txt" 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$ROOT/gpurun_out/pmc_$i" -o pmc \
    -- python3 "$ROOT/scripts/kbench.py" --reps 3 --only "$ONLY"
  rc=$?
  echo "pass $i rc=$rc"
  # unknown-counter errors are non-fatal; a timeout / crash ends the job
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
