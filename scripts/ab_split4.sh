#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "split" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/replay_probe.py > gpurun_out/replay_probe.log 2>&1
rc=$?; tail -1 gpurun_out/replay_probe.log; [ $rc -eq 0 ] || exit $rc
