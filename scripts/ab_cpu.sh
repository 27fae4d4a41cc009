#!/bin/bash
set -o pipefail
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
for cfg in "--cpu-workers 8" "--cpu-workers 16" "--cpu-workers 4"; do
  timeout -k 10 500 python bench.py --steps 3 --warmup 1 --verbose $cfg > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("engine",{}); print(d["value"], d["ms_per_step"], e.get("decode_steps"), e.get("decode_row_steps"), e.get("admit_s"), e.get("harvest_s"))')"
done
STEPS=2 MSGS=16384 bash scripts/gpu_prof.sh > gpurun_out/prof_run.log 2>&1; cat gpurun_out/prof/gaps.txt | head -8
