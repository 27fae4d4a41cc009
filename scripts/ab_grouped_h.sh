#!/bin/bash
# grouped decode attention vs grouped_h (per-sequence metadata hoisted to entry):
# numerics, per-op timing, interleaved bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attn" --timeout 120 --timeout-method thread > gpurun_out/gh_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gh_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 4096 8192; do
  timeout -k 10 300 python scripts/kbench.py --batch $B --ctx 72 > gpurun_out/gh_kbench_$B.json 2>gpurun_out/gh_kbench_$B.err
  rc=$?; python -c "import json,sys; d=json.loads(open('gpurun_out/gh_kbench_$B.json').read().strip().splitlines()[-1]); print($B, {k: d[k] for k in d if k.startswith('attn_decode_grouped')})"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for impl in grouped grouped_h; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --decode-attn $impl > gpurun_out/ab_gh_${impl}_$i.log 2>&1
    rc=$?; echo "$impl $i $(tail -1 gpurun_out/ab_gh_${impl}_$i.log | cut -c1-90)"; [ $rc -eq 0 ] || exit $rc
  done
done
