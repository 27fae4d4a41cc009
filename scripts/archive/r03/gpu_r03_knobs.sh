# Round-3 session 2: with 8 batches in flight per parser process, re-check the pipeline depth
# and the engine's chunking: interleaved A/B, two runs per arm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/r03s2_ab_knobs.jsonl --repeats 2 --timeout 500 \
  --arm "c8=" --arm "c16=--concurrency 16" --arm "spg3=--steps-per-graph 3" --arm "af25=--admit-frac 0.25" \
  --common=--verbose > gpurun_out/r03s2_ab_knobs.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_knobs.log; exit 1; }
tail -5 gpurun_out/r03s2_ab_knobs.log
