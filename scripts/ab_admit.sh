#!/bin/bash
# Headline bench, interleaved A/B: admission batching off (0) vs the default (32).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for mb in 0 32; do
    timeout -k 10 600 python bench.py --steps 5 --warmup 2 --admit-min-batch $mb > gpurun_out/ab_admit_${mb}_$i.log 2>&1
    rc=$?; echo "mb=$mb run $i: $(tail -1 gpurun_out/ab_admit_${mb}_$i.log | cut -c1-70)"; [ $rc -eq 0 ] || exit $rc
  done
done
