#!/bin/bash
# Round 5: parser processes per GPU A/B (the parsers ran at 7.0 of 8 cores at 65 k
# msgs/s), then what the QKV GEMM's RoPE / KV-scatter epilogue costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05o
mkdir -p $O
for w in 10 8 10 8; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose --cpu-workers $w --msgs-per-step 16000 \
    >> $O/workers_ab.jsonl 2>> $O/workers_ab.err || { echo "bench w=$w rc=$?"; tail -40 $O/workers_ab.err; exit 1; }
  tail -1 $O/workers_ab.jsonl | cut -c1-120
done
timeout -k 10 300 python -u scripts/qkv_epilogue_cost.py > $O/qkv_epi.jsonl 2> $O/qkv_epi.err \
  || { echo "qkv probe rc=$?"; tail -20 $O/qkv_epi.err; exit 1; }
cat $O/qkv_epi.jsonl
