#!/bin/bash
# per-op microbench at the speculative decode shapes (pseudo-rows per half batch)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 9216 4608; do
  timeout -k 10 400 python -u scripts/kbench.py --batch $B --ctx 60 > gpurun_out/kbench_b$B.json 2> gpurun_out/kbench_b$B.err
  rc=$?; tail -c 300 gpurun_out/kbench_b$B.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/kbench_b$B.err; exit $rc; }
done
