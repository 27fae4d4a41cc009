# Round-3 session 2: merged prefix + own key stream in the st attention kernels (GPU suite,
# then bench A/B interleaved: merged (default) vs --no-attn-merge, spec-frac 1.5), then a
# kernel profile of the default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 700 python -u bench.py --verbose "$@" > gpurun_out/ab4_$n.json 2> gpurun_out/ab4_$n.err || { tail -5 gpurun_out/ab4_$n.err; exit 1; }
  cut -c1-160 gpurun_out/ab4_$n.json
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "attn" > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run m1
run n1 --no-attn-merge
run m2
run n2 --no-attn-merge
run f150 --spec-frac 1.5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_m -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_m.log 2>&1) || { tail -5 gpurun_out/prof_m.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_m
find gpurun_out/prof_m -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_m/run_kernel_stats.csv > gpurun_out/prof_m/top.txt
head -16 gpurun_out/prof_m/top.txt
