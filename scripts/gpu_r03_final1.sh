# Round-3 session 2: GPU suite (QKV tile rule with the 4-wave 128x192 tile at decode halves),
# serving latency of the deployed latency profile and of the throughput profile (trained
# weights), the random-weights worst case, one default bench run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 700 python -u bench.py --verbose > gpurun_out/f1_bench.json 2> gpurun_out/f1_bench.err || { tail -5 gpurun_out/f1_bench.err; exit 1; }
cut -c1-200 gpurun_out/f1_bench.json
for prof in latency throughput; do
  timeout -k 10 400 python -u scripts/latency_bench.py --weights train --profile $prof --rates 1000,6000,10000,14000 --seconds 4 --out gpurun_out/r03s2_latency_$prof.json > gpurun_out/latency_$prof.log 2>&1 || { tail -5 gpurun_out/latency_$prof.log; exit 1; }
  grep offered gpurun_out/latency_$prof.log | cut -c1-160
done
timeout -k 10 600 python -u bench.py --weights random --eval-n 0 > gpurun_out/f1_random.json 2> gpurun_out/f1_random.err || { tail -5 gpurun_out/f1_random.err; exit 1; }
cut -c1-200 gpurun_out/f1_random.json
