#!/bin/bash
# Round 5: the whole GPU test suite and smoke() on the current tree (what the driver runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt | cut -c1-300
