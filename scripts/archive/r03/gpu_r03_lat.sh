# Round-3 session 2: serving latency of the revised latency profile (2 steps per graph, 12.5 %
# admission, 6 drafts, 4 096 rows) vs the round-2 one and the throughput profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > gpurun_out/lat_warm.log 2>&1 || { tail -3 gpurun_out/lat_warm.log; exit 1; }
for prof in latency latency_r2 throughput; do
  timeout -k 10 400 python -u scripts/latency_bench.py --weights train --profile $prof --rates 1000,6000,10000,14000 --seconds 4 --out gpurun_out/r03s2b_latency_$prof.json > gpurun_out/latb_$prof.log 2>&1 || { tail -5 gpurun_out/latb_$prof.log; exit 1; }
  grep offered gpurun_out/latb_$prof.log | cut -c1-120
done
