# Round-3 session 2: GPU suite (QKV tile rule with the 4-wave 128x192 tile at decode halves, sparse
# lm_head arg-max);
# interleaved A/B: sparse vs dense arg-max, parser priority, 12 288 slots; serving
# latency of the latency and throughput profiles (trained weights); random-weights worst case.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python -u scripts/ab.py --out gpurun_out/r03s2_ab_host.jsonl --repeats 2 --timeout 500 \
  --arm "base=" --arm "dense=--no-sparse-argmax" --arm "nice5=--worker-nice 5" --arm "ms12k=--max-slots 12288 --bucket-step 2048" \
  --common=--verbose > gpurun_out/r03s2_ab_host.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_host.log; exit 1; }
tail -5 gpurun_out/r03s2_ab_host.log
for prof in latency throughput; do
  timeout -k 10 400 python -u scripts/latency_bench.py --weights train --profile $prof --rates 1000,6000,10000,14000 --seconds 4 --out gpurun_out/r03s2_latency_$prof.json > gpurun_out/latency_$prof.log 2>&1 || { tail -5 gpurun_out/latency_$prof.log; exit 1; }
  grep offered gpurun_out/latency_$prof.log | cut -c1-160
done
timeout -k 10 600 python -u bench.py --weights random --eval-n 0 > gpurun_out/f1_random.json 2> gpurun_out/f1_random.err || { tail -5 gpurun_out/f1_random.err; exit 1; }
cut -c1-200 gpurun_out/f1_random.json
