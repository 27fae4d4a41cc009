#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_span_gpu.py -q --timeout 280 --timeout-method thread > gpurun_out/mask_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/mask_pytest.log; if [ $rc -ne 0 ]; then tail -30 gpurun_out/mask_pytest.log; exit 1; fi
bash scripts/gpu_r04_final.sh
