#!/bin/bash
# Round 5: qa decoder edges + time absorption (kernel vs reference), fused training
# kernels (fp32 references, A/B step time), then the GEMM SOL / split A/B of gpu_r05_d.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qa_gpu.py \
  tests/test_train_ops_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u scripts/train_step_profile.py --steps 40 > $O/train_step.jsonl 2> $O/train_step.err \
  || { echo "train profile rc=$?"; tail -30 $O/train_step.err; exit 1; }
cat $O/train_step.jsonl
bash scripts/gpu_r05_d.sh
