#!/bin/bash
# Split-decode at larger slot counts.
set -o pipefail
mkdir -p gpurun_out
for cfg in "--split-decode 4096" "--max-slots 16384 --msgs-per-step 32768 --split-decode 8192" "--max-slots 16384 --msgs-per-step 32768 --split-decode 4096" "--max-slots 16384 --msgs-per-step 32768" "--split-decode 4096 --steps-per-graph 4"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 $cfg > gpurun_out/ab_split2.log 2>&1 || { tail -5 gpurun_out/ab_split2.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab_split2.log | cut -c1-100)" | tee -a gpurun_out/ab_split2_summary.txt
done
