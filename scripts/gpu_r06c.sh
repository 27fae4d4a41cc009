#!/bin/bash
# round 6, call C: the persistent staggered residual GEMM (cfg 35-38) -- numerics first
# (bit-identical to cfg 28 / within rounding for the 32x32x16 A/B), then the interleaved
# tile sweep at the qa engine's shapes; then the qa engine's serving latency under
# Poisson arrivals for both profiles
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
if [ $rc -ne 0 ]; then exit $rc; fi
for prof in latency throughput; do
  timeout -k 10 240 python -u scripts/latency_bench.py --profile $prof --rates 1000,10000,40000 --seconds 6 \
    --out gpurun_out/r06_latency_qa_$prof.json > gpurun_out/r06c_latency_$prof.log 2>&1
  rc=$?
  echo "latency $prof rc=$rc"; tail -3 gpurun_out/r06c_latency_$prof.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
