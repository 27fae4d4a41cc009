# Counter passes for the gate_up GEMM (scripts/gemm_pmc.py); CFGS / B from the env.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
[ -f smsgate_amd/ops/_lib/libsmsgate_kernels.so ] || { echo "build the kernels first"; exit 1; }
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc -o q$i -- python $R/scripts/gemm_pmc.py > $R/gpurun_out/pmc/q$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc/q$i.log; exit 1; }
done
cd $R && python scripts/pmc_summary.py gpurun_out/pmc/q*_counter_collection.csv > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
