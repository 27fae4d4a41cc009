#!/bin/bash
# Round 5: prefill attention implementations at the qa engine's shapes (2 211 / 4 422
# packed sequences of 45-55 rows, shared prefix of 4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05dd
mkdir -p $O
timeout -k 10 300 python -u scripts/prefill_bench.py --nseq 2211,4422 --lens 45,56 --P0 4 --iters 30 \
  --out $O/prefill_qa.jsonl > $O/prefill.log 2>&1 || { echo "prefill rc=$?"; tail -30 $O/prefill.log; exit 1; }
cat $O/prefill_qa.jsonl
