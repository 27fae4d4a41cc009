#!/bin/bash
# Draft-budget / draft-length tuning of speculative decoding on the headline bench, plus training step time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/train_bench.py --batch 128 --steps 30 > gpurun_out/train_bench_b128.log 2>&1
rc=$?; tail -1 gpurun_out/train_bench_b128.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/ab_spec_tune2.jsonl --repeats 1 --common "--steps 10 --warmup 2 --eval-n 0" \
  --arm "k4f15=--spec-k 4 --spec-frac 1.5" --arm "k4f125=--spec-k 4 --spec-frac 1.25" --arm "k4f1=--spec-k 4 --spec-frac 1.0" --arm "k5f125=--spec-k 5 --spec-frac 1.25" --arm "k4f15b=--spec-k 4 --spec-frac 1.5"
