# Round-3 session 2: parser-side in-flight depth (--concurrency batches of 512 per parser
# process) vs the engine's waiting queue: interleaved A/B, three runs per arm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/r03s2_ab_conc.jsonl --repeats 3 --timeout 500 \
  --arm "c4=" --arm "c8=--concurrency 8" --common=--verbose > gpurun_out/r03s2_ab_conc.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_conc.log; exit 1; }
tail -4 gpurun_out/r03s2_ab_conc.log
