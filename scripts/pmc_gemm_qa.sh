#!/bin/bash
# Counter passes for the qa engine's big-M GEMMs (scripts/gemm_pmc.py at 110 592 rows):
# gate/up (persistent 256x256 SwiGLU, cfg 20), down-proj (K 1536) and o-proj (K 576) at
# 128x192 (cfg 28) and their old 96-wide tiles.  One counter set per run.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_qa
mkdir -p $O
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  for job in "swiglu 576 20" "resid 1536 28,21" "resid 576 28,22"; do
    set -- $job
    EPI=$1 K=$2 CFGS=$3 B=110592 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O -o q${i}_${1}_${2} \
      -- python $R/scripts/gemm_pmc.py > $O/q${i}_${1}_${2}.log 2>&1 || { echo "pass $i $job failed"; tail -5 $O/q${i}_${1}_${2}.log; exit 1; }
  done
done
cd $R && python scripts/pmc_summary.py --match gemm --by-grid gpurun_out/pmc_qa/q*_counter_collection.csv > gpurun_out/pmc_qa/summary.txt && cat gpurun_out/pmc_qa/summary.txt
