#!/bin/bash
# Training curves (135M flagship and the bundled small model) scored on held-out vocabulary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/train_curve.py --model smollm-135m --batch 128 --lr 1e-3 --steps 1500 --eval-every 250 > gpurun_out/curve_135m.log 2>&1
rc=$?; grep '"step"' gpurun_out/curve_135m.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/train_curve.py --model small --batch 128 --lr 2e-3 --steps 4000 --eval-every 1000 --out gpurun_out/extractor-small.safetensors > gpurun_out/curve_small.log 2>&1
rc=$?; grep '"step"' gpurun_out/curve_small.log | cut -c1-260; exit $rc
