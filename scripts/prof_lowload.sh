#!/bin/bash
# Kernel stats of the engine at low load (2k msgs/s Poisson): what sets the latency floor.
set -o pipefail
mkdir -p gpurun_out/prof_low
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_low -o run -- \
  python $GRAFT_REPO_ROOT/scripts/latency_bench.py --rates 2000 --seconds 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_low.log 2>&1
rc=$?; tail -2 $GRAFT_REPO_ROOT/gpurun_out/prof_low.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_low -name "*kernel_trace.csv" -size +20M -delete
exit $rc
