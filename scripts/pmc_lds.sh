#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $R/gpurun_out/pmc -o p3 -- python $R/scripts/gemm_pmc.py > $R/gpurun_out/pmc/p3.log 2>&1 || { tail $R/gpurun_out/pmc/p3.log; exit 1; }
python $R/scripts/pmc_summary.py $R/gpurun_out/pmc/p3_counter_collection.csv
