#!/bin/bash
# round 6, call R: kernel trace of the final engine (prefill attention auto = st32)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o final -- \
  python3 $GRAFT_REPO_ROOT/scripts/qa_engine_bench.py --n 65536 --reps 2 > $GRAFT_REPO_ROOT/$O/engine.json \
  2> $GRAFT_REPO_ROOT/$O/engine.err || { echo "rocprof rc=$?"; tail $GRAFT_REPO_ROOT/$O/engine.err; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/gpu_us_per_msg.py $O/prof/final_results.db --msgs 196608 --out $O/gpu_us_final.json
tail -c 600 $O/gpu_us_final.json
ls $O/prof
