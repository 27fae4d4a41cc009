# New tokenizer (number-aware pre-tokenizer): retrain the bundled small extractor and use
# it in place, GPU tests that depend on trained weights, the default bench, a profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 420 python -u scripts/quality_probe.py --model small --run '{"steps": 12000, "batch": 64, "lr": 0.002, "n_examples": 400000}' --save gpurun_out/extractor-small.safetensors --out gpurun_out/r03_quality_small3.jsonl > gpurun_out/r03_quality_small3.log 2>&1 || { tail -5 gpurun_out/r03_quality_small3.log; exit 1; }
cut -c1-400 gpurun_out/r03_quality_small3.jsonl
cp gpurun_out/extractor-small.safetensors smsgate_amd/models/assets/extractor-small.safetensors
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_llm_gpu.py tests/test_copy_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "template or golden or case or copy" > gpurun_out/r03_tok_pytest.log 2>&1 || { tail -30 gpurun_out/r03_tok_pytest.log; exit 1; }
tail -2 gpurun_out/r03_tok_pytest.log
timeout -k 10 600 python -u bench.py --verbose > gpurun_out/r03_bench_tok.json 2> gpurun_out/r03_bench_tok.err || { tail -5 gpurun_out/r03_bench_tok.err; exit 1; }
cut -c1-400 gpurun_out/r03_bench_tok.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_tok -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_tok.log 2>&1) || { tail -5 gpurun_out/prof_tok.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_tok
find gpurun_out/prof_tok -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_tok/run_kernel_stats.csv > gpurun_out/prof_tok/top.txt
