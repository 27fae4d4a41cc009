set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_spec_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "producer_norm or residual or measured or split_prefill or spec or template or store_and_norm" > gpurun_out/r03_k3.log 2>&1 || { tail -30 gpurun_out/r03_k3.log; exit 1; }
tail -2 gpurun_out/r03_k3.log
timeout -k 10 200 python -u scripts/gemm_tune.py --only down,o --rows 256,1024,1536,2048 --cfgs 3,17,18,21,22,27 --rounds 3 > gpurun_out/r03_small_tune.json 2> gpurun_out/r03_small_tune.err || { tail -5 gpurun_out/r03_small_tune.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03_small_tune.json'))
for k,v in d.items(): print(k, sorted(v['us'].items(), key=lambda x: x[1])[:6])"
