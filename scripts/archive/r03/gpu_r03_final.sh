# Round-3 session 2, final check of the committed tree: GPU suite, smoke, the driver's bench
# command, a kernel profile of the default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -5 gpurun_out/final_bench.err; exit 1; }
cut -c1-300 gpurun_out/final_bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_final.log 2>&1) || { tail -5 gpurun_out/prof_final.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_final
find gpurun_out/prof_final -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_final/run_kernel_stats.csv > gpurun_out/prof_final/top.txt
head -10 gpurun_out/prof_final/top.txt | cut -c1-120
