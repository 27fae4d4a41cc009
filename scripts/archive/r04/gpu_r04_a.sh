#!/bin/bash
# r04: span GPU tests (the template check included; failures recorded, not fatal), then the default bench
# (span, no templates) with CPU profiles + a rocprofv3 kernel-stats run
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_span_gpu.py -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/span_pytest2.log 2>&1
rc=$?; grep -E "PASS|FAIL|MISMATCH|TEMPLATES|passed|failed|^E " gpurun_out/span_pytest2.log | cut -c1-400 | tail -24
if [ $rc -gt 1 ]; then exit 1; fi
FMT=span bash $R/scripts/gpu_r04_bench.sh
