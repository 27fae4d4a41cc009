#!/bin/bash
# Round 5: BK 32 / 4-stage residual tiles (cfg 33, 34): numerics, then the residual
# tile sweep at the engine's row counts against cfg 28
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05bb
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "resid or tile or gemm" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/gemm_tune.py --rows 221184,110592,55296,27648 --only down,o \
  --cfgs 23,28,33,34 --rounds 3 --inner 8 > $O/gemm_tune.json 2> $O/gemm_tune.err \
  || { echo "gemm_tune rc=$?"; tail -20 $O/gemm_tune.err; exit 1; }
cat $O/gemm_tune.json
