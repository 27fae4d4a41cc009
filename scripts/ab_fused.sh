#!/bin/bash
# GPU suite + A/B of the headline bench: fused MFMA GEMMs vs hipBLASLt path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench_fused.log 2>&1
rc=$?; grep metric gpurun_out/bench_fused.log | cut -c1-200; [ $rc -eq 0 ] || { tail gpurun_out/bench_fused.log; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-fused-gemm > gpurun_out/bench_unfused.log 2>&1
rc=$?; grep metric gpurun_out/bench_unfused.log | cut -c1-200; exit $rc
