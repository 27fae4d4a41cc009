#!/bin/bash
# Round 5: trimmed last layer (GPU test), qa engine batch-size sweep, and where the
# training step's host-to-device copies come from.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qa_gpu.py \
  > $O/pytest_qa.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest_qa.log; exit 1; }
tail -3 $O/pytest_qa.log
timeout -k 10 400 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 \
  --qa-max-tokens 8192,16384,32768,65536,131072,262144 > $O/engine_sweep.jsonl 2> $O/engine_sweep.err \
  || { echo "engine rc=$?"; tail -20 $O/engine_sweep.err; exit 1; }
cut -c1-300 $O/engine_sweep.jsonl
timeout -k 10 300 python -u scripts/train_memcpy_probe.py > $O/memcpy.json 2> $O/memcpy.err \
  || { echo "memcpy probe rc=$?"; tail -20 $O/memcpy.err; exit 1; }
head -c 3000 $O/memcpy.json
