#!/bin/bash
# Round 5: fused training kernels (GPU tests), training-step SDPA backend A/B (fused on),
# then the qa-shape SOL table and the engine's two-stream split A/B (gpu_r05_d.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_ops_gpu.py \
  tests/test_qa_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for b in flash efficient; do
  SMSGATE_TRAIN_SDPA=$b timeout -k 10 300 python -u scripts/train_step_profile.py --steps 40 --fused 1 \
    > $O/train_step_$b.jsonl 2> $O/train_step_$b.err || { echo "train profile $b rc=$?"; tail -30 $O/train_step_$b.err; exit 1; }
  cut -c1-400 $O/train_step_$b.jsonl
done
O_D=$O bash scripts/gpu_r05_d.sh
