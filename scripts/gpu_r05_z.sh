#!/bin/bash
# Round 5: the whole GPU suite on the final tree, then the driver's bench twice
# (per-connection sender threads, parse-time zone check, DDP sample alignment)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose >> $O/bench.jsonl 2>> $O/bench.err \
    || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-200
done
