#!/bin/bash
# Full GPU suite + smoke + training throughput + 2 headline bench runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/train_bench.py --out gpurun_out/train_bench.json > gpurun_out/train_bench.log 2>&1
rc=$?; tail -1 gpurun_out/train_bench.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_full$i.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_full$i.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
