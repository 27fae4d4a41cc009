#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "--split-graphs 1" "--split-graphs 2" "--split-graphs 1" "--split-graphs 2"; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --verbose $cfg > gpurun_out/ab_split5.log 2>&1 || { tail -5 gpurun_out/ab_split5.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab_split5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["engine"]; print(d["value"], "decode_s", e["decode_s"], "admit_s", e["admit_s"], "harvest_wait_s", e["harvest_wait_s"], "step_s", e["step_s"], "poll", e["server_poll_s"])')" | tee -a gpurun_out/ab_split5_summary.txt
done
