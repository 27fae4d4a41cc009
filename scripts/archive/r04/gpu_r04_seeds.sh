#!/bin/bash
# r04: seed spread of the span model at the bench's recipe (4000 steps x 128, lr 1e-3)
set -o pipefail
mkdir -p gpurun_out
for s in 1 2; do
  timeout -k 10 540 python -u scripts/family_probe.py --steps 4000 --batch 128 --lr 1e-3 --seed $s --eval-every 0 \
    --format span --tag r4_seed$s --jsonl gpurun_out/family_probe_seeds.jsonl > gpurun_out/probe_seed$s.log 2>&1 \
    || { tail -5 gpurun_out/probe_seed$s.log; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/family_probe_seeds.jsonl'):
    d=json.loads(l); print(d['tag'], d['step'], d['train_s'], d['heldout_formats']['exact'], d['heldout_formats']['by_family'], d['train_formats']['exact'], d['legacy_mix_exact'], d['cases_mismatches'])"
