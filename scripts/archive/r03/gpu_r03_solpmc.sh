#!/bin/bash
# measured HBM bytes of the speed-of-light cases: FETCH_SIZE and WRITE_SIZE passes (one
# counter group per run), every case launched 5 times directly
set -o pipefail
mkdir -p gpurun_out/solpmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/solpmc -o p$i -- python $R/scripts/sol_table.py --direct 5 > $R/gpurun_out/solpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/solpmc/p$i.log; exit 1; }
done
cd $R && python scripts/pmc_summary.py --by-grid --match "" gpurun_out/solpmc/p*_counter_collection.csv > gpurun_out/solpmc/summary.txt && cat gpurun_out/solpmc/summary.txt && tail -1 gpurun_out/solpmc/p1.log
