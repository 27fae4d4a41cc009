#!/bin/bash
# Round 5: training-step SDPA backend A/B (fused kernels on), then the qa-shape SOL
# table and the engine's two-stream split A/B (gpu_r05_d.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05f
mkdir -p $O
for b in flash efficient; do
  SMSGATE_TRAIN_SDPA=$b timeout -k 10 300 python -u scripts/train_step_profile.py --steps 40 --fused 1 \
    > $O/train_step_$b.jsonl 2> $O/train_step_$b.err || { echo "train profile $b rc=$?"; tail -30 $O/train_step_$b.err; exit 1; }
  cat $O/train_step_$b.jsonl
done
O_D=$O bash scripts/gpu_r05_d.sh
