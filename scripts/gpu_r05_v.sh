#!/bin/bash
# Round 5: what the QKV+RoPE epilogue costs at the engine's layout (packed sequences)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 python -u scripts/qkv_epilogue_cost.py > $O/qkv_epi.jsonl 2> $O/qkv_epi.err \
  || { echo "qkv probe rc=$?"; tail -20 $O/qkv_epi.err; exit 1; }
cat $O/qkv_epi.jsonl
