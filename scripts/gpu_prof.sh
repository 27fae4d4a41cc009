#!/bin/bash
# Kernel-level profile of the headline bench (kernel trace + stats only; no PMC).
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-2} --warmup 1 --msgs-per-step ${MSGS:-2048} ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -40 "$f" | cut -c1-250
t=$(find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*kernel_trace.csv" | head -1)
[ -n "$t" ] && python $GRAFT_REPO_ROOT/scripts/trace_gaps.py "$t" > $GRAFT_REPO_ROOT/gpurun_out/prof/gaps.txt 2>&1; cat $GRAFT_REPO_ROOT/gpurun_out/prof/gaps.txt
# keep the merged output small: drop the big per-dispatch trace
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete
exit $rc
