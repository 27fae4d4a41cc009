# Round-3 session 2: are the two-stream halves still worth it now that attention is cheaper?
# prefill as one batch (--split-prefill 0), decode as one batch (--split-decode 0), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/r03s2_ab_split.jsonl --repeats 2 --timeout 500 \
  --arm "base=" --arm "sp0=--split-prefill 0" --arm "sd0=--split-decode 0" --common=--verbose > gpurun_out/r03s2_ab_split.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_split.log; exit 1; }
tail -4 gpurun_out/r03s2_ab_split.log
