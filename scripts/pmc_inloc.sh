#!/bin/bash
# PMC counter passes over the InLoc pipeline (bench_inloc.py), one counter
# group per rocprofv3 run, kernels matching $2 only -> gpurun_out/pmcinl_<pass>/
#   scripts/pmc_inloc.sh SIZE REGEX [extra bench_inloc args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE="${1:-3200}"; RX="${2:-corr_gemm}"
shift $(( $# > 2 ? 2 : $# ))
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf "$ROOT/gpurun_out/pmcinl_$i"
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d "$ROOT/gpurun_out/pmcinl_$i" -o pmc \
    -- python3 "$ROOT/scripts/bench_inloc.py" --image-size "$SIZE" --pairs 2 --warmup 1 "$@"
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
