#!/bin/bash
# Round 5: engine batch policy A/B end to end (sender thread in the engine server):
# a second in-flight batch only after 64 k queued rows vs immediately.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05m
mkdir -p $O
for mt in 65536 0; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose --qa-min-tokens $mt \
    >> $O/policy_ab.jsonl 2>> $O/policy_ab.err || { echo "bench mt=$mt rc=$?"; tail -40 $O/policy_ab.err; exit 1; }
  tail -1 $O/policy_ab.jsonl | cut -c1-120
done
