#!/bin/bash
# Round 5: training tests after the host-side loss denominator, then the driver's bench
# (quality must match the r05s run family for family: the training stream is unchanged)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py \
  tests/test_train_ops_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
