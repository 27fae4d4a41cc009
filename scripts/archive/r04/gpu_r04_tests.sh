#!/bin/bash
# r04: the whole GPU suite (every failure listed, not just the first) + smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25
if [ $rc -gt 1 ]; then exit 1; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-300
