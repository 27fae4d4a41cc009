#!/bin/bash
# Round 5: GEMM / attention speed-of-light at the qa format's shapes, and the engine's
# two-stream split A/B (one prefill of the whole batch vs two concurrent halves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=${O_D:-gpurun_out/r05d}
mkdir -p $O
timeout -k 10 300 python -u scripts/sol_table.py --no-spec --decode-m 221184 --prefill-m 110592 --prefill-len 50 \
  --rounds 2 > $O/sol.json 2> $O/sol.err || { echo "sol rc=$?"; tail -20 $O/sol.err; exit 1; }
cat $O/sol.json
for r in 1 2; do
  for sp in 8192 0; do
    timeout -k 10 240 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 --split-prefill $sp \
      >> $O/split_ab.jsonl 2>> $O/split_ab.err || { echo "engine rc=$?"; tail -20 $O/split_ab.err; exit 1; }
  done
done
cat $O/split_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o nosplit -- python3 scripts/qa_engine_bench.py \
  --n 65536 --reps 2 --split-prefill 0 > $O/engine_nosplit.json 2> $O/engine_nosplit.err \
  || { echo "rocprof rc=$?"; tail $O/engine_nosplit.err; exit 1; }
python scripts/gpu_us_per_msg.py $O/prof/nosplit_results.db --msgs 196608 --out $O/gpu_us_nosplit.json
