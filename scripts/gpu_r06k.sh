#!/bin/bash
# round 6, call K: QKV+RoPE configs at the engine's packed layout (cfg 39 = 40 + 41)
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 300 python -u scripts/qkv_packed_tune.py --rows 110592 > $O/packed.json 2> $O/packed.err \
  || { echo "rc=$?"; tail -5 $O/packed.err; exit 1; }
timeout -k 10 300 python -u scripts/qkv_packed_tune.py --rows 55296 >> $O/packed.json 2>> $O/packed.err \
  || { echo "rc=$?"; tail -5 $O/packed.err; exit 1; }
cat $O/packed.json
