#!/bin/bash
# Round 5: tile change + non-spinning engine: GPU tests, engine throughput, then two
# training-length variants of the qa probe (fused training kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qa_gpu.py \
  tests/test_kernels_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 > $O/engine.json 2> $O/engine.err \
  || { echo "engine rc=$?"; tail -20 $O/engine.err; exit 1; }
cat $O/engine.json
timeout -k 10 900 python -u scripts/qa_probe.py --formats qa --eval-n 1000 --variants "steps=4000;steps=6000" \
  --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -30 $O/probe.log; exit 1; }
cut -c1-600 $O/probe.jsonl
