#!/bin/bash
# Training curves of the 135M flagship (two batch/lr settings) scored on held-out vocabulary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/train_curve.py --model smollm-135m --batch 128 --lr 1e-3 --steps 1500 --eval-every 300 > gpurun_out/curve2_135m_b128.log 2>&1
rc=$?; grep -E '"step"|step  *[0-9]+00 ' gpurun_out/curve2_135m_b128.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/train_curve.py --model smollm-135m --batch 256 --lr 1.5e-3 --steps 900 --eval-every 300 > gpurun_out/curve2_135m_b256.log 2>&1
rc=$?; grep -E '"step"|step  *[0-9]+00 ' gpurun_out/curve2_135m_b256.log | cut -c1-200; exit $rc
