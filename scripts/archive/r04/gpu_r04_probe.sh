#!/bin/bash
# r04: small bundled asset on the new tokenizer + a 135M held-out-family probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u scripts/family_probe.py --model small --steps 12000 --batch 64 --lr 2e-3 --examples 400000 \
  --eval-every 0 --tag small_r4g --jsonl gpurun_out/family_probe_small.jsonl --out gpurun_out/extractor-small.safetensors \
  > gpurun_out/probe_small.log 2>&1 || { tail -5 gpurun_out/probe_small.log; exit 1; }
timeout -k 10 600 python -u scripts/family_probe.py --steps 3000 --batch 128 --lr 1e-3 --seed 0 --eval-every 1500 --tag r4g \
  > gpurun_out/probe_r4g.log 2>&1 || { tail -5 gpurun_out/probe_r4g.log; exit 1; }
