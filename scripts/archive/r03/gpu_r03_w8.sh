#!/bin/bash
# 8-wave 96-wide residual tiles (cfg 30 / 31): correctness, then an interleaved sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "producer_norm" > gpurun_out/r03s3_w8_pytest.txt 2>&1 && tail -2 gpurun_out/r03s3_w8_pytest.txt &&
timeout -k 10 400 python -u scripts/gemm_tune.py --rows 4608,9216,15104 --only down,o --cfgs 21,22,30,31 --rounds 6 > gpurun_out/r03s3_w8_tune.json 2> gpurun_out/r03s3_w8_tune.log && cat gpurun_out/r03s3_w8_tune.json
