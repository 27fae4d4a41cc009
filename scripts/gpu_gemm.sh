#!/bin/bash
# Fused GEMM bring-up: numerics first (own timeout), then the GPU suite, microbench, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -k gemm -x -q -p no:cacheprovider > gpurun_out/pytest_gemm.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --batch 4096 --ctx 75 > gpurun_out/kbench.json 2> gpurun_out/kbench.err
rc=$?; cat gpurun_out/kbench.json; [ $rc -eq 0 ] || { tail gpurun_out/kbench.err; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench.log 2>&1
rc=$?; grep metric gpurun_out/bench.log | cut -c1-600; exit $rc
