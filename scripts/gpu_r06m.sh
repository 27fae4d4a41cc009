#!/bin/bash
# round 6, call M: prefill attention variants at the qa engine's packed batches (P0 = 4
# prefix tokens, ~53-row messages): st64 (the auto choice from 1 024 sequences) against
# st64 with the one-tile register prefetch (st64pf) and the 32-column forms
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python -u scripts/prefill_bench.py --nseq 1044,2089,4178 --lens 40,67 --P0 4 --iters 30 \
  --impls st32,st64,st32pf,st64pf --out $O/prefill.jsonl > $O/prefill.log 2>&1 || { echo "rc=$?"; tail -5 $O/prefill.log; exit 1; }
cat $O/prefill.jsonl
