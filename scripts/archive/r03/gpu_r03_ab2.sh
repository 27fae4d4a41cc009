# Template KV reuse with the copy kernel, and a 16 384-row engine, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "kv_copy or template" > gpurun_out/r03_tpl2_pytest.log 2>&1 || { tail -30 gpurun_out/r03_tpl2_pytest.log; exit 1; }
tail -2 gpurun_out/r03_tpl2_pytest.log
timeout -k 10 900 python -u scripts/ab.py --out gpurun_out/r03_ab_templates2.jsonl --repeats 2 --timeout 400 --arm "tpl0=--template-slots 0" --arm "tpl16=--template-slots 16" --arm "tpl16_16k=--template-slots 16 --max-slots 16384" --common "--steps 12 --warmup 2 --verbose" > gpurun_out/r03_ab_templates2.log 2>&1
rc=$?; tail -8 gpurun_out/r03_ab_templates2.log; exit $rc
