#!/bin/bash
# GPU test suite (one process), first the files named in $1 (if any), then everything.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest $1 -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_first.log 2>&1
  rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu_first.log | tail -30; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; exit $rc
