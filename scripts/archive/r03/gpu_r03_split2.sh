# Round-3 session 2: confirm prefill as one batch (--split-prefill 0) vs two halves, 3 runs each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/r03s2_ab_split2.jsonl --repeats 3 --timeout 500 \
  --arm "base=" --arm "sp0=--split-prefill 0" --common=--verbose > gpurun_out/r03s2_ab_split2.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_split2.log; exit 1; }
tail -3 gpurun_out/r03s2_ab_split2.log
