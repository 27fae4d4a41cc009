#!/bin/bash
# Kernel tests for the prefill change + prefill microbench + short headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_prefill.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_prefill.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/prefill_bench.py --out gpurun_out/prefill_bench.json > gpurun_out/prefill_bench.log 2>&1
rc=$?; tail -3 gpurun_out/prefill_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench2.log 2>&1
rc=$?; tail -1 gpurun_out/bench2.log | cut -c1-400; exit $rc
