#!/bin/bash
# Round 5: training attention kernels (tests + step A/B), qa engine batch-size sweep
# (activations resident in the 256 MB Infinity Cache vs spilling to HBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_ops_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u scripts/train_step_profile.py --steps 40 --fused 1 > $O/train_step.jsonl 2> $O/train_step.err \
  || { echo "train profile rc=$?"; tail -30 $O/train_step.err; exit 1; }
cut -c1-500 $O/train_step.jsonl
timeout -k 10 400 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 \
  --qa-max-tokens 8192,16384,24576,32768,49152,65536,131072,262144 > $O/engine_sweep.jsonl 2> $O/engine_sweep.err \
  || { echo "engine rc=$?"; tail -20 $O/engine_sweep.err; exit 1; }
cut -c1-260 $O/engine_sweep.jsonl
