#!/bin/bash
# Shared-broker vs in-process bus on the headline bench (spec on), then serving latency with/without spec.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in "--bus busd" "--bus memory" "--bus busd" "--bus memory"; do
  tag=$(echo $arm | tr -d ' -')
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --verbose --eval-n 0 --spec-k 4 $arm > gpurun_out/busab_$tag.log 2>&1
  rc=$?; tail -1 gpurun_out/busab_$tag.log | cut -c1-140; [ $rc -eq 0 ] || exit $rc
done
for k in 0 4; do
  timeout -k 10 400 python -u scripts/latency_bench.py --weights train --spec-k $k --rates 1000,2000,6000,10000 --seconds 4 --out gpurun_out/latency_spec$k.json > gpurun_out/latency_spec$k.log 2>&1
  rc=$?; grep offered gpurun_out/latency_spec$k.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
