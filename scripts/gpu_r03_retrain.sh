# Retrain the bundled small extractor (tokenization changed: &#10; -> one token, <sms> in the
# shared prefix), then the default bench (in-run 135M training) with --verbose.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u scripts/quality_probe.py --model small --run '{"steps": 12000, "batch": 64, "lr": 0.002, "n_examples": 400000}' --save gpurun_out/extractor-small.safetensors --out gpurun_out/r03_quality_small2.jsonl > gpurun_out/r03_quality_small2.log 2>&1 || { tail -5 gpurun_out/r03_quality_small2.log; exit 1; }
cut -c1-400 gpurun_out/r03_quality_small2.jsonl
timeout -k 10 600 python -u bench.py --verbose > gpurun_out/r03_bench2.json 2> gpurun_out/r03_bench2.err
rc=$?; cut -c1-300 gpurun_out/r03_bench2.json; exit $rc
