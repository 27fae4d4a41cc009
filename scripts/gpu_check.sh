#!/bin/bash
# First-contact GPU run: kernel/engine numerics, smoke, short bench. Each GPU step has its own timeout.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== rocm-smi"; (rocm-smi --showproductname 2>&1 | head -20) || true
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; cat gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; exit $rc
