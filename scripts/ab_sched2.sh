#!/bin/bash
set -o pipefail
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
for cfg in "--steps-per-graph 2" "--steps-per-graph 3" "--steps-per-graph 4" "--steps-per-graph 6" "--admit-frac 0.15" "--admit-frac 0.35" "--max-slots 6144" "--max-slots 8192 --msgs-per-step 16384"; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --verbose $cfg > gpurun_out/ab.log 2>&1 || exit 1
  echo "[$cfg] $(grep metric gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("engine",{}); print(d["value"], d["ms_per_step"], e.get("decode_steps"), e.get("decode_row_steps"))')"
done
