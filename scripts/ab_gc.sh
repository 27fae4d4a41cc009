#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "--no-gc-freeze" "" "--no-gc-freeze" "" "--no-gc-freeze" ""; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 $cfg > gpurun_out/ab_gc.log 2>&1 || { tail -5 gpurun_out/ab_gc.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab_gc.log | cut -c1-100)" | tee -a gpurun_out/ab_gc_summary.txt
done
