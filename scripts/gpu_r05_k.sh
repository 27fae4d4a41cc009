#!/bin/bash
# Round 5: the driver's bench command on the current tree, and the training step's
# host-to-device copies traced to their CPU ops.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench failed rc=$?"; tail -40 $O/bench.err; exit 1; }
tail -c 1200 $O/bench.json
timeout -k 10 300 python -u scripts/train_memcpy_probe.py > $O/memcpy.json 2> $O/memcpy.err \
  || { echo "memcpy probe rc=$?"; tail -20 $O/memcpy.err; exit 1; }
head -c 3000 $O/memcpy.json
