#!/bin/bash
# Headline bench with in-run trained weights, then a longer small-model training for the bundled checkpoint.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py --steps 10 --warmup 2 --verbose > gpurun_out/bench_v2.log 2>&1
rc=$?; tail -2 gpurun_out/bench_v2.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/train_curve.py --model small --batch 128 --lr 2e-3 --steps 12000 --eval-every 4000 --out gpurun_out/extractor-small.safetensors > gpurun_out/curve2_small.log 2>&1
rc=$?; grep '"step"' gpurun_out/curve2_small.log | cut -c1-400; exit $rc
