#!/bin/bash
# Final-defaults evidence: full GPU suite, smoke, latency sweep, headline bench x2
# and a kernel-stats profile of the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/latency_bench.py --rates 1000,2000,6000,10000,14000 --seconds 4 --out gpurun_out/latency_final.json > gpurun_out/lat_final.log 2>&1
rc=$?; grep offered gpurun_out/lat_final.log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_final$i.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_final$i.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_final -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_final.log 2>&1
rc=$?; tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof_final.log | cut -c1-120
find $GRAFT_REPO_ROOT/gpurun_out/prof_final -name "*kernel_trace.csv" -size +20M -delete
exit $rc
