#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "split" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_split.log; [ $rc -eq 0 ] || exit $rc
for cfg in "" "--split-parts 3" "--split-parts 4" "" "--split-parts 3" "--split-parts 4"; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 $cfg > gpurun_out/ab_split6.log 2>&1 || { tail -5 gpurun_out/ab_split6.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab_split6.log | cut -c1-100)" | tee -a gpurun_out/ab_split6_summary.txt
done
