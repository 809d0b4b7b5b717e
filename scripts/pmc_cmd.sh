#!/bin/bash
# Two PMC counter passes (one counter group per rocprofv3 run) over any python
# command; CSVs under gpurun_out/pmc_<tag>_<pass>/.
#   scripts/pmc_cmd.sh <tag> <script.py> [args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
cd /tmp
export TMPDIR=/tmp PYTHONPATH="$ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
# PMC_L2=1: a third pass with the L2 hit / miss / HBM read-request counters
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
PASSES=("$P1" "$P2")
[ "${PMC_L2:-0}" = 1 ] && PASSES+=("$P3")
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$ROOT/gpurun_out/pmc_${TAG}_$i" -o pmc \
    -- python3 "$@"
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
DIRS=()
for j in $(seq 1 $i); do DIRS+=("$ROOT/gpurun_out/pmc_${TAG}_$j"); done
python3 "$ROOT/scripts/pmc_summary.py" "${DIRS[@]}" \
  --out "$ROOT/gpurun_out/pmc_${TAG}.md"
