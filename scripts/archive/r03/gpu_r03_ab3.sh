# Round-3 session 2: draft budget vs GEMM tile rounds (1.25 B -> 9 216-row halves = 1.69 rounds of
# 256x256 gate/up tiles, 1.5 B -> 10 240 rows = 1.88 rounds), interleaved, then a kernel profile
# of the default with the transposed prefill attention.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 700 python -u bench.py --verbose "$@" > gpurun_out/ab3_$n.json 2> gpurun_out/ab3_$n.err || { tail -5 gpurun_out/ab3_$n.err; exit 1; }
  cut -c1-200 gpurun_out/ab3_$n.json
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run def1
run f150 --spec-frac 1.5
run def2
run f100 --spec-frac 1.0
run f150b --spec-frac 1.5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_st -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_st.log 2>&1) || { tail -5 gpurun_out/prof_st.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_st
find gpurun_out/prof_st -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_st/run_kernel_stats.csv > gpurun_out/prof_st/top.txt
head -20 gpurun_out/prof_st/top.txt
