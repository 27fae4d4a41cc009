#!/bin/bash
# Round 5: kernel tests after the V^T chunk change, the QKV GEMM at the qa shapes, and
# the driver's bench command twice on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_qa_gpu.py -k "qkv or qa" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/qkv_epilogue_cost.py > $O/qkv_epi.jsonl 2> $O/qkv_epi.err \
  || { echo "qkv probe rc=$?"; tail -20 $O/qkv_epi.err; exit 1; }
grep -v skip $O/qkv_epi.jsonl
for r in 1 2; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose >> $O/bench.jsonl 2>> $O/bench.err \
    || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-120
done
