set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_abi.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "prefill or residual or producer_norm or measured or abi or qkv" > gpurun_out/r03_k2.log 2>&1 || { tail -20 gpurun_out/r03_k2.log; exit 1; }
tail -2 gpurun_out/r03_k2.log
timeout -k 10 120 python -u scripts/prefill_bench.py --out gpurun_out/r03_prefill_bench.jsonl > gpurun_out/r03_prefill_bench.log 2>&1 || { tail -5 gpurun_out/r03_prefill_bench.log; exit 1; }
cat gpurun_out/r03_prefill_bench.jsonl | cut -c1-400
timeout -k 10 200 python -u scripts/gemm_tune.py --only qkv_rope --rows 4608,9216,16384 --rounds 3 > gpurun_out/r03_qkv_tune.json 2> gpurun_out/r03_qkv_tune.err || { tail -5 gpurun_out/r03_qkv_tune.err; exit 1; }
tail -c 800 gpurun_out/r03_qkv_tune.json
timeout -k 10 900 python -u scripts/ab.py --out gpurun_out/r03_ab_resid_prefill.jsonl --repeats 2 --timeout 400 --arm "base=--no-resid96" --arm "resid96=" --arm "resid96_multi=--prefill-attn multi" --common "--steps 12 --warmup 2 --eval-n 0" > gpurun_out/r03_ab_resid_prefill.log 2>&1
rc=$?; tail -8 gpurun_out/r03_ab_resid_prefill.log; exit $rc
