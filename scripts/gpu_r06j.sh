#!/bin/bash
# round 6, call J: cfg 39 (persistent QK+RoPE + cfg-28 V) numerics against cfg 28, the
# existing QKV tests, then its timing at the qa shapes (sol_table's QKV row per cfg)
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "qk_rope_persistent or qkv or producer_norm" > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u scripts/gemm_tune.py --rows 110592,55296 --only qkv_rope --cfgs 28,39 --rounds 3 \
  > $O/tune.json 2> $O/tune.err || { echo "tune rc=$?"; tail -5 $O/tune.err; exit 1; }
cat $O/tune.json
