#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over one kbench case:
#   scripts/pmc_one.sh <kbench case> <out dir under gpurun_out> [vols]
# pass 1: wave-state split, pass 2: MFMA / LDS / clock, pass 3: L2 hit / miss.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CASE="$1"; OUT="$ROOT/gpurun_out/$2"; VOLS="${3:-64}"
cd /tmp
export TMPDIR=/tmp PYTHONPATH="$ROOT"
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pass$i" -o pmc \
    -- python3 "$ROOT/scripts/kbench.py" --reps 3 --vols "$VOLS" --only "$CASE" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pass1" "$OUT/pass2" "$OUT/pass3" > "$OUT/summary.md" 2>&1 || true
