#!/bin/bash
# Fused InLoc NC kernel: oracle tests, then the 3200 px volume timing (+ PMC pass)
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "nc_fused or fused_symmetric" > gpurun_out/ncf_tests.log 2>&1 || exit $?
timeout -k 10 120 python scripts/nc_fused_bench.py --reps 20 > gpurun_out/ncf_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
rm -rf "$R/gpurun_out/pmcnc_x"
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex nc_fused --output-format csv -d "$R/gpurun_out/pmcnc_x" -o pmc -- python3 "$R/scripts/nc_fused_bench.py" --reps 3 > /dev/null 2>&1 || exit $?
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmcnc_x" --out "$R/gpurun_out/pmc_ncfused_x.md"
