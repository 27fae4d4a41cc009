#!/bin/bash
# Round 5: error analysis + profiles of the qa default (bench with cProfile, errors of
# the trained weights, kernel stats of the engine alone, the training step's time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --verbose --profile-cpu $O/cprof \
  > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -30 $O/bench.err; exit 1; }
python scripts/cprof_top.py $O/cprof --bench $O/bench.json > $O/cprof_top.txt 2>&1 || true
timeout -k 10 180 python -u scripts/qa_errors.py > $O/errors.jsonl 2> $O/errors.err || { echo "errors rc=$?"; tail $O/errors.err; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o qa -- python3 scripts/qa_engine_bench.py --n 65536 --reps 2 \
  > $O/engine_bench.json 2> $O/engine_bench.err || { echo "rocprof rc=$?"; tail $O/engine_bench.err; exit 1; }
timeout -k 10 240 python -u scripts/train_step_profile.py > $O/train_step.json 2> $O/train_step.err || { echo "train prof rc=$?"; tail $O/train_step.err; }
cat $O/engine_bench.json $O/train_step.json
