#!/bin/bash
# Counter passes + kernel trace for the decode attention (scripts/attn_pmc.py):
# HBM bytes fetched vs the bytes it must read, L2 hit rate, wave occupancy.
set -o pipefail
mkdir -p gpurun_out/pmc_attn
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for B in 4096 8192; do
  export B
  timeout -k 10 120 python $R/scripts/attn_pmc.py > $R/gpurun_out/pmc_attn/shape_$B.json || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_attn -o kt$B -- python $R/scripts/attn_pmc.py > $R/gpurun_out/pmc_attn/kt$B.log 2>&1 || { tail -5 $R/gpurun_out/pmc_attn/kt$B.log; exit 1; }
  i=0
  for set in "FETCH_SIZE GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_attn -o b${B}_p$i -- python $R/scripts/attn_pmc.py > $R/gpurun_out/pmc_attn/b${B}_p$i.log 2>&1 || { echo "B=$B pass $i failed"; tail -5 $R/gpurun_out/pmc_attn/b${B}_p$i.log; exit 1; }
  done
done
cd $R && python scripts/pmc_summary.py --match attn gpurun_out/pmc_attn/b*_counter_collection.csv > gpurun_out/pmc_attn/summary.txt; cat gpurun_out/pmc_attn/summary.txt
