#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_span_gpu.py -q --timeout 400 --timeout-method thread \
  > gpurun_out/span_pytest4.log 2>&1 || { tail -30 gpurun_out/span_pytest4.log; exit 1; }
tail -1 gpurun_out/span_pytest4.log
bash scripts/gpu_r04_rankthr.sh
