#!/bin/bash
# Headline bench, interleaved A/B: tokenizer threads per parser process (0 = one per CPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
for i in 1 2; do
  for t in 0 2 4; do
    timeout -k 10 600 python bench.py --steps 5 --warmup 2 --worker-threads $t > gpurun_out/ab_threads_${t}_$i.log 2>&1
    rc=$?; echo "threads=$t run $i: $(tail -1 gpurun_out/ab_threads_${t}_$i.log | cut -c1-70)"; [ $rc -eq 0 ] || exit $rc
  done
done
