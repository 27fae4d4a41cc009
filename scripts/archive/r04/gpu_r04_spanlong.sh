#!/bin/bash
# r04: does longer training close the span format's held-out gap (97.4 % vs copy 99.2 %)?
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/family_probe.py --steps 5000 --batch 128 --lr 1e-3 --seed 0 --eval-every 1000 \
  --format span --tag r4h_span5k --jsonl gpurun_out/family_probe_span5k.jsonl > gpurun_out/probe_span5k.log 2>&1 \
  || { tail -5 gpurun_out/probe_span5k.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/family_probe_span5k.jsonl'):
    d=json.loads(l); print(d['step'], d['train_s'], d['heldout_formats']['exact'], d['heldout_formats']['by_family'], d['train_formats']['exact'], d['legacy_mix_exact'], d['cases_mismatches'])"
