#!/bin/bash
# Counter passes: cfg 28 (128x192, 2 blocks per CU) against cfg 35 (persistent staggered 256x192)
# for the residual GEMMs at 110 592 rows: down-proj (K 1536) and o-proj (K 576).
# One counter set per run.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_r06
mkdir -p $O
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  for job in "resid 1536 28,35" "resid 576 28,35"; do
    set -- $job
    EPI=$1 K=$2 CFGS=$3 B=110592 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O -o q${i}_${1}_${2} \
      -- python $R/scripts/gemm_pmc.py > $O/q${i}_${1}_${2}.log 2>&1 || { echo "pass $i $job failed"; tail -5 $O/q${i}_${1}_${2}.log; exit 1; }
  done
done
cd $R && python scripts/pmc_summary.py --match gemm --by-grid gpurun_out/pmc_r06/q*_counter_collection.csv > gpurun_out/pmc_r06/summary.txt && cat gpurun_out/pmc_r06/summary.txt
