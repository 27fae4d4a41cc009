#!/bin/bash
# round 6, call G: the smoke test (bundled qa extractor: CASE 1 + a rejected held-out
# non-transaction), the headline bench as the driver runs it (in-run training with the
# round-6 recipe, the quality gates on), and a kernel trace of the engine alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
  || { echo "smoke rc=$?"; tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt | cut -c1-400
timeout -k 10 900 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o final -- \
  python3 $GRAFT_REPO_ROOT/scripts/qa_engine_bench.py --n 65536 --reps 2 > $GRAFT_REPO_ROOT/$O/engine.json \
  2> $GRAFT_REPO_ROOT/$O/engine.err || { echo "rocprof rc=$?"; tail $GRAFT_REPO_ROOT/$O/engine.err; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/gpu_us_per_msg.py $O/prof/final_results.db --msgs 196608 --out $O/gpu_us_final.json
tail -c 600 $O/gpu_us_final.json
