#!/bin/bash
# grouped6 (grouped decode attention at 6 waves/SIMD, 80 VGPRs): numerics, per-op
# timing at the large buckets, interleaved headline A/B against grouped.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k "attn_decode" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn2.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_attn2.log; [ $rc -eq 0 ] || exit $rc
for b in 4096 8192; do
  timeout -k 10 300 python scripts/kbench.py --batch $b --ctx 72 > gpurun_out/kbench_g6_b$b.json 2> gpurun_out/kbench_g6_b$b.err
  rc=$?; echo "kbench $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for impl in grouped grouped6; do
    timeout -k 10 600 python bench.py --steps 5 --warmup 2 --decode-attn $impl > gpurun_out/ab_g6_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i: $(tail -1 gpurun_out/ab_g6_${impl}_$i.log | cut -c1-70)"; [ $rc -eq 0 ] || exit $rc
  done
done
