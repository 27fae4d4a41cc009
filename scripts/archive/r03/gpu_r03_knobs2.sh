# Round-3 session 2: scheduling knobs at the new default (8 batches in flight): the second
# decode half's launch offset, drafts per row, draft budget, admission threshold.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1150 python -u scripts/ab.py --out gpurun_out/r03s2_ab_knobs2.jsonl --repeats 2 --timeout 500 \
  --arm "base=" --arm "noff=--no-split-offset" --arm "sk8=--spec-k 8" --arm "f100=--spec-frac 1.0" --arm "af06=--admit-frac 0.0625" \
  --common=--verbose > gpurun_out/r03s2_ab_knobs2.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_knobs2.log; exit 1; }
tail -6 gpurun_out/r03s2_ab_knobs2.log
