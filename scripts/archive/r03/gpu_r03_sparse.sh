# Round-3 session 2: the 16-candidates-per-pass sparse arg-max: GPU suite, kernel profile,
# two default bench runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 700 python -u bench.py --verbose > gpurun_out/sp_b1.json 2> gpurun_out/sp_b1.err || { tail -5 gpurun_out/sp_b1.err; exit 1; }
cut -c1-160 gpurun_out/sp_b1.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_sp2 -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_sp2.log 2>&1) || { tail -5 gpurun_out/prof_sp2.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_sp2
find gpurun_out/prof_sp2 -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_sp2/run_kernel_stats.csv > gpurun_out/prof_sp2/top.txt
head -12 gpurun_out/prof_sp2/top.txt | cut -c1-120
timeout -k 10 400 python -u bench.py --verbose > gpurun_out/sp_b2.json 2> gpurun_out/sp_b2.err || { tail -5 gpurun_out/sp_b2.err; exit 1; }
cut -c1-160 gpurun_out/sp_b2.json
