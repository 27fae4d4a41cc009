#!/bin/bash
# Steady-state (20 timed steps) re-check of scheduling knobs swept earlier at 5 steps.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "" "--steps-per-graph 4" "--admit-frac 0.35" "--cpu-workers 16"; do
    tag=$(echo "x$cfg" | tr -c 'a-z0-9\n' '_')
    timeout -k 10 300 python bench.py $cfg > gpurun_out/ab_steady_${tag}_$i.log 2>&1
    rc=$?; echo "[$cfg] $i $(tail -1 gpurun_out/ab_steady_${tag}_$i.log | cut -c40-75)"; [ $rc -eq 0 ] || exit $rc
  done
done
