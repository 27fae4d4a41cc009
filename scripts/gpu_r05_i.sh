#!/bin/bash
# Round 5: placement A/B on the 1-GPU box: the default bench with
# --pin on / off, interleaved (the first run trains and caches the weights).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05i
mkdir -p $O
for pin in on off on off; do
  timeout -k 10 900 python -u bench.py --steps 10 --warmup 2 --pin $pin >> $O/pin_ab.jsonl 2>> $O/pin_ab.err \
    || { echo "bench pin=$pin rc=$?"; tail -30 $O/pin_ab.err; exit 1; }
  tail -1 $O/pin_ab.jsonl | cut -c1-200
done
