#!/bin/bash
# Counter passes for the prefill attention (scripts/prefill_pmc.py): issue vs wait.
set -o pipefail
mkdir -p gpurun_out/pmc_prefill
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for IMPL in per_head multi; do
  export IMPL
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_prefill -o kt_$IMPL -- python $R/scripts/prefill_pmc.py > $R/gpurun_out/pmc_prefill/kt_$IMPL.log 2>&1 || { tail -5 $R/gpurun_out/pmc_prefill/kt_$IMPL.log; exit 1; }
  i=0
  for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
             "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_prefill -o ${IMPL}_p$i -- python $R/scripts/prefill_pmc.py > $R/gpurun_out/pmc_prefill/${IMPL}_p$i.log 2>&1 || { echo "$IMPL pass $i failed"; tail -5 $R/gpurun_out/pmc_prefill/${IMPL}_p$i.log; exit 1; }
  done
done
cd $R && python scripts/pmc_summary.py --match prefill gpurun_out/pmc_prefill/*_counter_collection.csv > gpurun_out/pmc_prefill/summary.txt; cat gpurun_out/pmc_prefill/summary.txt
