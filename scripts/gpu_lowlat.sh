#!/bin/bash
# Low-load latency work: GPU suite, per-op timings at small decode buckets, and a
# latency A/B (grouped attention + 64-row GEMM tiles vs key-split attention +
# 32-row GEMM tiles on small buckets), then the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for b in 256 512 1024 2048 4096; do
  timeout -k 10 300 python scripts/kbench.py --batch $b --ctx 72 > gpurun_out/kbench_b$b.json 2> gpurun_out/kbench_b$b.err
  rc=$?; echo "kbench $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/latency_bench.py --rates 2000,6000,10000 --seconds 3 --attn-small-rows 0 --gemm-small-m 0 > gpurun_out/lat_base.log 2>&1
rc=$?; tail -3 gpurun_out/lat_base.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/latency_bench.py --rates 2000,6000,10000 --seconds 3 --attn-small-rows 1024 --gemm-small-m 1024 > gpurun_out/lat_small.log 2>&1
rc=$?; tail -3 gpurun_out/lat_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?; tail -1 gpurun_out/bench1.log | cut -c1-200; exit $rc
