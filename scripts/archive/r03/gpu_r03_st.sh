# Round-3 session 2: health check of the tree (GPU suite, smoke) + the transposed
# register prefill attention kernel (microbench, then bench A/B: st32 vs auto).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 200 python -u scripts/prefill_bench.py --nseq 150,300,800 --out gpurun_out/r03_prefill_st.jsonl > gpurun_out/prefill_st.log 2>&1 || { tail -5 gpurun_out/prefill_st.log; exit 1; }
cut -c1-600 gpurun_out/r03_prefill_st.jsonl
timeout -k 10 700 python -u bench.py --verbose --cases-required 0 > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err || { tail -5 gpurun_out/bench_auto.err; exit 1; }
cut -c1-300 gpurun_out/bench_auto.json; grep "CASES" gpurun_out/bench_auto.err
timeout -k 10 400 python -u bench.py --verbose --cases-required 0 --prefill-attn st32 > gpurun_out/bench_st32.json 2> gpurun_out/bench_st32.err || { tail -5 gpurun_out/bench_st32.err; exit 1; }
cut -c1-300 gpurun_out/bench_st32.json
timeout -k 10 400 python -u bench.py --verbose --cases-required 0 > gpurun_out/bench_auto2.json 2> gpurun_out/bench_auto2.err || { tail -5 gpurun_out/bench_auto2.err; exit 1; }
cut -c1-300 gpurun_out/bench_auto2.json
timeout -k 10 400 python -u bench.py --verbose --cases-required 0 --prefill-attn st > gpurun_out/bench_st.json 2> gpurun_out/bench_st.err || { tail -5 gpurun_out/bench_st.err; exit 1; }
cut -c1-300 gpurun_out/bench_st.json
