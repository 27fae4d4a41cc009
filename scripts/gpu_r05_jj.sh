#!/bin/bash
# Round 5: the driver's bench on the final tree (engine-server sender guard)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05jj
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
