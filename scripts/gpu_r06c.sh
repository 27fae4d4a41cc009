#!/bin/bash
# round 6, call C: the persistent staggered residual GEMM (cfg 35-38) -- numerics first
# (bit-identical to cfg 28 / within rounding for the 32x32x16 A/B), then the interleaved
# tile sweep at the qa engine's shapes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "resid_persistent or residual_inplace or producer_norm" > gpurun_out/r06c_pytest_gemm.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r06c_pytest_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 python -u scripts/gemm_tune.py --rows 110592,55296,27648 --only down,o --cfgs 28,35,36,37,38 \
  --rounds 3 > gpurun_out/r06c_gemm_tune.json 2> gpurun_out/r06c_gemm_tune.err
rc=$?
echo "tune rc=$rc"; cat gpurun_out/r06c_gemm_tune.json
exit $rc
