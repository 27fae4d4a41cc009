#!/bin/bash
# Longer-run A/B for grouped_h (15 timed steps per run, arm order alternating per pair).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then arms="grouped grouped_h"; else arms="grouped_h grouped"; fi
  for impl in $arms; do
    timeout -k 10 300 python bench.py --steps 15 --warmup 2 --decode-attn $impl > gpurun_out/ab_gh3_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i $(tail -1 gpurun_out/ab_gh3_${impl}_$i.log | cut -c1-90)"; [ $rc -eq 0 ] || exit $rc
  done
done
