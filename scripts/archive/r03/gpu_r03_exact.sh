# Round-3 session 2: exact-key loads in the merged attention tiles (GPU suite, two default
# bench runs, kernel profile).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 700 python -u bench.py --verbose "$@" > gpurun_out/ab6_$n.json 2> gpurun_out/ab6_$n.err || { tail -5 gpurun_out/ab6_$n.err; exit 1; }
  cut -c1-160 gpurun_out/ab6_$n.json
}
run d1
run d2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ex -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_ex.log 2>&1) || { tail -5 gpurun_out/prof_ex.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_ex
find gpurun_out/prof_ex -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_ex/run_kernel_stats.csv > gpurun_out/prof_ex/top.txt
head -12 gpurun_out/prof_ex/top.txt
