#!/bin/bash
# Round 5: prefill attention auto = 64 columns from 1 024 sequences: bitwise test, the
# attention / engine / qa tests, then the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05ee
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_prefill" > $O/pytest_attn.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qa_gpu.py \
  tests/test_engine_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
