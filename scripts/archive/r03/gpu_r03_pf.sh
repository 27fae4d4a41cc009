#!/bin/bash
# prefill attention with the one-tile register prefetch (st32pf / stpf): correctness, microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r03s3_pf_pytest.txt 2>&1 && tail -2 gpurun_out/r03s3_pf_pytest.txt &&
timeout -k 10 300 python -u scripts/prefill_bench.py --nseq 200,408,800 --lens 30,45 --P0 4 --out gpurun_out/r03s3_prefill_pf.jsonl > gpurun_out/r03s3_prefill_pf.log 2>&1 && cat gpurun_out/r03s3_prefill_pf.jsonl
