#!/bin/bash
# Scheduling A/B: decode bucket granularity and admission threshold.
set -o pipefail
mkdir -p gpurun_out
for cfg in "" "--bucket-step 1024" "--bucket-step 512" "--admit-frac 0.125" "--admit-frac 0.125 --bucket-step 1024" ""; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 $cfg > gpurun_out/ab4.log 2>&1 || { tail -5 gpurun_out/ab4.log; exit 1; }
  echo "[$cfg] $(grep metric gpurun_out/ab4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("engine",{}); print(d["value"], d["ms_per_step"], e.get("decode_steps"), e.get("decode_row_steps"), round(e.get("decode_row_steps",0)/max(1,e.get("decode_steps",1))), e.get("prefill_seqs"))')" | tee -a gpurun_out/ab4_summary.txt
done
