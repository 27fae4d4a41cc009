# Round-3 session 2: kernel profiles of the default (sparse lm_head arg-max) and of the dense
# arg-max, same trained weights.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 700 python -u bench.py --steps 2 --warmup 1 > gpurun_out/prof2_warm.log 2>&1 || { tail -3 gpurun_out/prof2_warm.log; exit 1; }
for arm in sparse dense; do
  extra=""; [ $arm = dense ] && extra="--no-sparse-argmax"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$arm -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 $extra > $R/gpurun_out/prof_$arm.log 2>&1) || { tail -5 gpurun_out/prof_$arm.log; exit 1; }
  python scripts/prof_summary.py gpurun_out/prof_$arm
  find gpurun_out/prof_$arm -name "*kernel_trace.csv" -delete
  python scripts/stats_top.py gpurun_out/prof_$arm/run_kernel_stats.csv > gpurun_out/prof_$arm/top.txt
  head -14 gpurun_out/prof_$arm/top.txt | cut -c1-120
done
