#!/bin/bash
# grouped_pf (prefetching grouped decode attention): numerics, per-op timing at the
# large decode buckets, and an interleaved headline A/B against grouped.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k "attn_decode" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
for b in 2048 4096 8192; do
  timeout -k 10 300 python scripts/kbench.py --batch $b --ctx 72 > gpurun_out/kbench_pf_b$b.json 2> gpurun_out/kbench_pf_b$b.err
  rc=$?; echo "kbench $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for impl in grouped grouped_pf; do
    timeout -k 10 600 python bench.py --steps 5 --warmup 2 --decode-attn $impl > gpurun_out/ab_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i: $(tail -1 gpurun_out/ab_${impl}_$i.log | cut -c1-80)"; [ $rc -eq 0 ] || exit $rc
  done
done
