#!/bin/bash
# Round 5: GEMM tile sweep at the qa engine's prefill-half shapes, then one bench with
# the CPU sampling profile of every process (parser workers + rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u scripts/gemm_tune.py --rows 110592,55296 --rounds 2 --inner 8 > $O/gemm_tune.json \
  2> $O/gemm_tune.err || { echo "gemm_tune rc=$?"; tail -20 $O/gemm_tune.err; exit 1; }
cat $O/gemm_tune.json
SMSGATE_TRAIN_SDPA=math timeout -k 10 300 python -u scripts/train_step_profile.py --steps 40 --fused 1 \
  > $O/train_step_math.jsonl 2> $O/train_step_math.err || { echo "train profile math rc=$?"; tail -30 $O/train_step_math.err; exit 1; }
cut -c1-400 $O/train_step_math.jsonl
timeout -k 10 900 python -u bench.py --steps 10 --warmup 2 --profile-cpu $O/sprof ${BENCH_ARGS} \
  > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -40 $O/bench.err; exit 1; }
python scripts/samples_top.py $O/sprof --bench $O/bench.json -n 40 > $O/samples_top.txt
timeout -k 10 300 python -u scripts/qa_errors.py --n 600 --per-family 8 > $O/errors.jsonl 2> $O/errors.err \
  || { echo "qa_errors rc=$?"; tail -20 $O/errors.err; }
tail -c 1500 $O/bench.json
