#!/bin/bash
# cfg 42 (gate/up with both A register sets) vs cfg 20: equality + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "two_a_sets or swiglu" > gpurun_out/r06p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06p_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_tune.py --only gate_up --cfgs 20,42 --rows 110592,55296,27648 \
  > gpurun_out/r06p_gemm_tune.json 2> gpurun_out/r06p_gemm_tune.err
rc=$?; echo "tune rc=$rc"; cat gpurun_out/r06p_gemm_tune.json
exit $rc
