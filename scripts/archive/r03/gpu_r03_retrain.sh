# Retrain the bundled small extractor (tokenization changed: &#10; -> one token, <sms> in the
# shared prefix) and use it in place, then the template tests, then an interleaved bench A/B
# of the message-start template KV reuse (in-run 135M training).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u scripts/quality_probe.py --model small --run '{"steps": 12000, "batch": 64, "lr": 0.002, "n_examples": 400000}' --save gpurun_out/extractor-small.safetensors --out gpurun_out/r03_quality_small2.jsonl > gpurun_out/r03_quality_small2.log 2>&1 || { tail -5 gpurun_out/r03_quality_small2.log; exit 1; }
cut -c1-300 gpurun_out/r03_quality_small2.jsonl
cp gpurun_out/extractor-small.safetensors smsgate_amd/models/assets/extractor-small.safetensors
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_llm_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "template or golden or case" > gpurun_out/r03_tpl_pytest.log 2>&1 || { tail -30 gpurun_out/r03_tpl_pytest.log; exit 1; }
tail -2 gpurun_out/r03_tpl_pytest.log
timeout -k 10 800 python -u scripts/ab.py --out gpurun_out/r03_ab_templates.jsonl --repeats 2 --timeout 400 --arm "tpl0=--template-slots 0" --arm "tpl16=--template-slots 16" --common "--steps 12 --warmup 2 --verbose" > gpurun_out/r03_ab_templates.log 2>&1
rc=$?; tail -6 gpurun_out/r03_ab_templates.log; exit $rc
