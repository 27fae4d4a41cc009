#!/bin/bash
# Round 5: edge rules of the qa decoder -- kernel vs reference tests, then a quality probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qa_gpu.py \
  > $O/qa_pytest.log 2>&1 || { echo "qa pytest failed rc=$?"; tail -30 $O/qa_pytest.log; exit 1; }
tail -3 $O/qa_pytest.log
timeout -k 10 900 python -u scripts/qa_probe.py --formats ${FORMATS:-qa} --steps ${STEPS:-4000} --eval-n 1000 \
  --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo "probe failed rc=$?"; tail -30 $O/probe.log; exit 1; }
tail -2 $O/probe.log
