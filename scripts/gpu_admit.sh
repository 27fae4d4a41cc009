#!/bin/bash
# Admission batching at low load: engine tests, then an interleaved latency A/B
# (admit every chunk vs hold arrivals for a bigger prefill).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_engine2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_engine2.log; [ $rc -eq 0 ] || exit $rc
for arm in "0 10" "32 10" "64 20" "128 20"; do
  set -- $arm
  timeout -k 10 300 python scripts/latency_bench.py --rates 1000,2000,6000 --seconds 3 --admit-min-batch $1 --admit-max-wait-ms $2 > gpurun_out/lat_admit_$1_$2.log 2>&1
  rc=$?; grep offered gpurun_out/lat_admit_$1_$2.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
