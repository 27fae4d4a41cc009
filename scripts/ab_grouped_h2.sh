#!/bin/bash
# Confirmation A/B for grouped_h, arm order reversed (grouped_h first in each pair).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for impl in grouped_h grouped; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --decode-attn $impl > gpurun_out/ab_gh2_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i $(tail -1 gpurun_out/ab_gh2_${impl}_$i.log | cut -c1-90)"; [ $rc -eq 0 ] || exit $rc
  done
done
