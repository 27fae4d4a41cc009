#!/bin/bash
# Round 5: the whole GPU suite and the driver's smoke on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest rc=$?"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
  || { echo "smoke rc=$?"; tail -30 $O/smoke.txt; exit 1; }
tail -5 $O/smoke.txt
