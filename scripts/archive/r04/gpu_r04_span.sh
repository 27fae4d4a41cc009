#!/bin/bash
# r04: span-pointer format kernels / engine / learning test, the small bundled asset (copy
# format) on the new tokenizer, and a 135M held-out-family probe in span format
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_span_gpu.py -v --timeout 400 --timeout-method thread \
  > gpurun_out/span_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/span_pytest.log
# test failures (1) do not stop the probes; a crash, hang or timeout does
if [ $rc -gt 1 ]; then exit 1; fi
timeout -k 10 300 python -u scripts/family_probe.py --model small --steps 12000 --batch 64 --lr 2e-3 --examples 400000 \
  --eval-every 0 --tag small_r4g --jsonl gpurun_out/family_probe_small.jsonl --out gpurun_out/extractor-small.safetensors \
  > gpurun_out/probe_small.log 2>&1 || { tail -5 gpurun_out/probe_small.log; exit 1; }
timeout -k 10 480 python -u scripts/family_probe.py --steps 3000 --batch 128 --lr 1e-3 --seed 0 --eval-every 1500 \
  --format span --tag r4g_span > gpurun_out/probe_r4g_span.log 2>&1 || { tail -5 gpurun_out/probe_r4g_span.log; exit 1; }
