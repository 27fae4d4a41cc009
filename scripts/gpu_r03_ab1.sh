set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_abi.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "prefill or residual or producer_norm or measured or abi" > gpurun_out/r03_k2.log 2>&1 || { tail -20 gpurun_out/r03_k2.log; exit 1; }
tail -2 gpurun_out/r03_k2.log
timeout -k 10 120 python -u scripts/prefill_bench.py --out gpurun_out/r03_prefill_bench.jsonl > gpurun_out/r03_prefill_bench.log 2>&1 || { tail -5 gpurun_out/r03_prefill_bench.log; exit 1; }
cat gpurun_out/r03_prefill_bench.jsonl | cut -c1-400
timeout -k 10 1000 python -u scripts/ab.py --out gpurun_out/r03_ab_resid_prefill.jsonl --repeats 2 --timeout 400 --arm "base=--no-resid96" --arm "resid96=" --arm "resid96_multi=--prefill-attn multi" --common "--steps 12 --warmup 2 --eval-n 0" > gpurun_out/r03_ab_resid_prefill.log 2>&1
rc=$?; tail -8 gpurun_out/r03_ab_resid_prefill.log; exit $rc
