set -u
timeout -k 10 300 python scripts/bench_inloc.py --image-size 3200 --pairs 10 --warmup 2 --panos-per-query 10 --precision bf16 > gpurun_out/inloc3200.log 2>&1 || exit $?
bash scripts/prof_inloc.sh 3200 _r4 --panos-per-query 10 --precision bf16 || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf "$R/gpurun_out/pmcnc_$i"
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex nc_fused --output-format csv -d "$R/gpurun_out/pmcnc_$i" -o pmc -- python3 "$R/scripts/nc_fused_bench.py" --reps 3 || exit $?
done
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmcnc_1" "$R/gpurun_out/pmcnc_2" --out "$R/gpurun_out/pmc_ncfused_r4.md"
