#!/bin/bash
# r04 final tree: the whole GPU suite + smoke, then serving latency (span answers, trained weights)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
if [ $rc -gt 1 ]; then exit 1; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 700 python -u scripts/latency_bench.py --weights train --profile latency --rates 1000,6000,10000,14000 \
  --seconds 4 --out gpurun_out/r04_latency_span.json > gpurun_out/r04_latency_span.log 2>&1 \
  || { tail -5 gpurun_out/r04_latency_span.log; exit 1; }
grep offered gpurun_out/r04_latency_span.log | cut -c1-200
