#!/bin/bash
# round 6, call N: the qa engine alone with each prefill attention form (auto = st64 at
# these batch sizes, st32, st32pf), interleaved, auto repeated last
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 --prefill-attn auto,st32,st32pf,auto \
  > $O/engine.jsonl 2> $O/engine.err || { echo "rc=$?"; tail -5 $O/engine.err; exit 1; }
cat $O/engine.jsonl
