#!/bin/bash
# Interleaved bench A/B: grouped decode attention (default) vs the key-split
# kernel at every bucket size (more, shorter waves to interleave with the other
# half-batch's GEMMs).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for impl in grouped split2; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --decode-attn $impl > gpurun_out/ab_attnall_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i $(tail -1 gpurun_out/ab_attnall_${impl}_$i.log | cut -c1-90)"; [ $rc -eq 0 ] || exit $rc
  done
done
