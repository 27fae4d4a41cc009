#!/bin/bash
# Confirm the small-bucket defaults: engine GPU tests, latency under Poisson load,
# a kernel-stats profile at 2k msgs/s (what sets the low-load floor now), and
# the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_engine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/latency_bench.py --rates 1000,2000,6000,10000,14000 --seconds 4 --out gpurun_out/latency_defaults.json > gpurun_out/lat_defaults.log 2>&1
rc=$?; tail -5 gpurun_out/lat_defaults.log; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_lowload.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1
rc=$?; tail -1 gpurun_out/bench2.log | cut -c1-200; exit $rc
