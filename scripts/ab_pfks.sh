#!/bin/bash
# Key-split prefill attention: numerics, microbench at serving shapes (small and
# large prefill batches), latency A/B at low load, interleaved headline A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k "attn_prefill" --timeout 120 --timeout-method thread > gpurun_out/pytest_prefill.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_prefill.log; [ $rc -eq 0 ] || exit $rc
for n in 32 190 800; do
  timeout -k 10 120 python scripts/prefill_bench.py --nseq $n > gpurun_out/prefill_ks_$n.json 2>&1
  rc=$?; tail -1 gpurun_out/prefill_ks_$n.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
for ks in 1 2; do
  timeout -k 10 300 python scripts/latency_bench.py --rates 1000,2000,6000 --seconds 3 --prefill-key-split $ks > gpurun_out/lat_pfks_$ks.log 2>&1
  rc=$?; grep offered gpurun_out/lat_pfks_$ks.log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for ks in 1 2; do
    timeout -k 10 600 python bench.py --steps 5 --warmup 2 --prefill-key-split $ks > gpurun_out/ab_pfks_${ks}_$i.log 2>&1
    rc=$?; echo "ks=$ks $i: $(tail -1 gpurun_out/ab_pfks_${ks}_$i.log | cut -c1-70)"; [ $rc -eq 0 ] || exit $rc
  done
done
