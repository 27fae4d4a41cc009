#!/bin/bash
# Round 5: occupancy 2 for the 128x192 residual / QKV GEMMs (residual chunks loaded after
# the K loop, cos/sin shared by the heads of a QKV tile): kernel + qa tests, the tile
# sweep at the qa shapes, the engine alone, then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_qa_gpu.py tests/test_ops_abi.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/gemm_tune.py --rows 110592,55296 --rounds 2 --inner 8 > $O/gemm_tune.json \
  2> $O/gemm_tune.err || { echo "gemm_tune rc=$?"; tail -20 $O/gemm_tune.err; exit 1; }
cat $O/gemm_tune.json | cut -c1-3000
timeout -k 10 300 python -u scripts/sol_table.py --no-spec --decode-m 221184 --prefill-m 110592 --prefill-len 50 \
  > $O/sol.json 2> $O/sol.err || { echo "sol rc=$?"; tail -20 $O/sol.err; exit 1; }
timeout -k 10 240 python -u scripts/qa_engine_bench.py --n 65536 --reps 3 > $O/engine.json 2> $O/engine.err \
  || { echo "engine rc=$?"; tail -20 $O/engine.err; exit 1; }
tail -2 $O/engine.json
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
