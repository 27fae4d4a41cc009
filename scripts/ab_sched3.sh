#!/bin/bash
set -o pipefail
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
for cfg in "--max-slots 8192 --msgs-per-step 16384 --steps-per-graph 2" "--max-slots 12288 --msgs-per-step 24576 --steps-per-graph 2" "--max-slots 16384 --msgs-per-step 32768 --steps-per-graph 2" "--max-slots 16384 --msgs-per-step 32768 --steps-per-graph 4" "--max-slots 16384 --msgs-per-step 32768 --steps-per-graph 2 --cpu-workers 12"; do
  timeout -k 10 500 python bench.py --steps 3 --warmup 1 --verbose $cfg > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("engine",{}); print(d["value"], d["ms_per_step"], e.get("decode_steps"), e.get("decode_row_steps"), e.get("admit_s"), e.get("harvest_s"))')"
done
