#!/bin/bash
# Round 5: the qa format on the GPU -- kernel / engine tests, then one short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05qa
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qa_gpu.py \
  > $O/qa_pytest.log 2>&1 || { echo "qa pytest failed rc=$?"; tail -30 $O/qa_pytest.log; exit 1; }
tail -3 $O/qa_pytest.log
timeout -k 10 720 python -u bench.py --steps ${STEPS:-10} --warmup 2 --verbose ${BENCH_ARGS} \
  > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -40 $O/bench.err; exit 1; }
cat $O/bench.json
