#!/bin/bash
# round 6, call E: the restructured persistent staggered residual GEMM (tile loop with a
# clean K loop: no per-step accumulator copies; residual requested on a tile's last
# K-step) -- numerics vs cfg 28, then the interleaved tile sweep at the qa shapes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "resid_persistent or residual_inplace or producer_norm" > gpurun_out/r06e_pytest_gemm.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06e_pytest_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 python -u scripts/gemm_tune.py --rows 110592,55296,27648 --only down,o --cfgs 28,35,36,37,38 \
  --rounds 3 > gpurun_out/r06e_gemm_tune.json 2> gpurun_out/r06e_gemm_tune.err
rc=$?
echo "tune rc=$rc"; cat gpurun_out/r06e_gemm_tune.json
exit $rc
