#!/bin/bash
# round 6, call T: engine batch size at the final kernels (bigger packed batches)
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 400 python -u scripts/qa_engine_bench.py --n 131072 --reps 2 --prefill-attn auto \
  --request 512 --max-slots 8192 --qa-max-tokens 262144 > $O/base.jsonl 2> $O/base.err \
  || { echo "base rc=$?"; tail -5 $O/base.err; exit 1; }
cat $O/base.jsonl
timeout -k 10 400 python -u scripts/qa_engine_bench.py --n 131072 --reps 2 --prefill-attn auto \
  --request 1024 --max-slots 16384 --qa-max-tokens 262144,524288 > $O/big.jsonl 2> $O/big.err \
  || { echo "big rc=$?"; tail -5 $O/big.err; exit 1; }
cat $O/big.jsonl
