#!/bin/bash
# Round 5: kernel trace of the bench's timed bus phase (random weights: no in-run training
# in the trace; the GPU work per message is the same), to compare the kernels' time per
# message with the engine alone (r05_qa_nosplit_kernel_stats.csv)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 10 \
  --warmup 2 --weights random --quality-floor 0 --cases-required 0 --false-parse-ceiling 1 --eval-n 0 --ingest bus \
  --verbose > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
find $O/prof -name "*kernel_stats.csv" | head -3
