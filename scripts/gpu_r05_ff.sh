#!/bin/bash
# Round 5: GEMM rasterisation group at the qa shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05ff
mkdir -p $O
timeout -k 10 300 python -u scripts/group_m_sweep.py 110592 > $O/group_m.jsonl 2> $O/group_m.err \
  || { echo "sweep rc=$?"; tail -20 $O/group_m.err; exit 1; }
cat $O/group_m.jsonl
