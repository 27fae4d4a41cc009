#!/bin/bash
# Round 5: the bench with engine statistics per phase (--verbose) after the batch policy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose > $O/bench.json 2> $O/bench.err \
  || { echo "bench failed rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -c 2500 $O/bench.json
