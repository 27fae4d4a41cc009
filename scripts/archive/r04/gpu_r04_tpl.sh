#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_span_gpu.py -v -s --timeout 380 --timeout-method thread \
  -k "templates or learns" > gpurun_out/span_tpl.log 2>&1
rc=$?; tail -30 gpurun_out/span_tpl.log; if [ $rc -gt 1 ]; then exit 1; fi
