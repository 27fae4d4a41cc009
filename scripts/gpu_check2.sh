#!/bin/bash
# new-kernel tests first, then the whole GPU suite, smoke, and the headline bench with new defaults
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spec_gpu.py tests/test_golden_llm_gpu.py tests/test_engine_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_new.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --verbose > gpurun_out/bench_defaults.log 2>&1
rc=$?; tail -1 gpurun_out/bench_defaults.log | cut -c1-2500; exit $rc
