#!/bin/bash
# Round 5 final: the whole GPU suite and the driver's smoke on the final tree, then a
# kernel trace of the engine alone for the final kernel mix and GPU us per message
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05gg
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
  || { echo "smoke rc=$?"; tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o final -- python3 scripts/qa_engine_bench.py \
  --n 65536 --reps 2 > $O/engine.json 2> $O/engine.err || { echo "rocprof rc=$?"; tail $O/engine.err; exit 1; }
python scripts/gpu_us_per_msg.py $O/prof/final_results.db --msgs 196608 --out $O/gpu_us_final.json
tail -c 600 $O/gpu_us_final.json
