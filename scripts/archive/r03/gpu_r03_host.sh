# Round-3 session 2: GPU idle between engine steps follows host CPU contention; interleaved A/B of
# the rank process's torch threads and the parser processes' priority.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1150 python -u scripts/ab.py --out gpurun_out/r03s2_ab_host.jsonl --repeats 2 --timeout 500 \
  --arm "base=" --arm "rt2=--rank-threads 2" --arm "nice5=--worker-nice 5" --arm "both=--rank-threads 2 --worker-nice 5" --arm "ms12k=--max-slots 12288 --bucket-step 2048" \
  --common "--verbose" > gpurun_out/r03s2_ab_host.log 2>&1
rc=$?; tail -8 gpurun_out/r03s2_ab_host.log; exit $rc
