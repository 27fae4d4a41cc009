#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
python -m smsgate_amd.ops.build >/dev/null 2>&1 || exit 1
for cfg in "--steps-per-graph 8" "--steps-per-graph 4" "--steps-per-graph 4 --admit-frac 0.125 --bucket-step 512" "--steps-per-graph 8 --admit-frac 0.125 --bucket-step 512" "--steps-per-graph 4 --admit-frac 0.06 --bucket-step 256"; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --verbose $cfg > gpurun_out/ab.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/ab.log; exit 1; }
  echo "$cfg :: $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"decode_row_steps": [0-9]*' gpurun_out/ab.log) $(grep -o '"decode_steps": [0-9]*' gpurun_out/ab.log)"
done
