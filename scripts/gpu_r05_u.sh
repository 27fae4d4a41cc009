#!/bin/bash
# Round 5: the 256x192 8-wave residual tile (cfg 32): its numerics tests, then an
# interleaved sweep of the residual tiles at the engine's row counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "resid or tile or gemm" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/gemm_tune.py --rows 221184,110592,55296,27648 --only down,o \
  --cfgs 21,22,23,28,30,32 --rounds 3 --inner 8 > $O/gemm_tune.json 2> $O/gemm_tune.err \
  || { echo "gemm_tune rc=$?"; tail -20 $O/gemm_tune.err; exit 1; }
cat $O/gemm_tune.json
