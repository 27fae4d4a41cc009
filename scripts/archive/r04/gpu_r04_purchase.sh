#!/bin/bash
# r04: span answers on round 3's traffic (purchase), for the like-for-like GPU time per
# message against profiles/r03s3_final_kernel_stats.csv (36.8 us, copy answers)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py --traffic purchase --steps 20 --warmup 2 --ingest bus --verbose \
  > gpurun_out/purchase.json 2> gpurun_out/purchase.err || { tail -20 gpurun_out/purchase.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/purchase.json') if l.startswith('{')][-1])
print('value', d['value'], d['routing'], d['quality_heldout']['legacy_mix']['exact'], d['quality_heldout']['reference_cases'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_purchase -o run -- python3 $R/bench.py \
  --traffic purchase --steps 10 --warmup 2 --eval-n 0 --quality-floor 0 --ingest bus \
  > $R/gpurun_out/purchase_prof.json 2> $R/gpurun_out/purchase_prof.err || { tail -20 $R/gpurun_out/purchase_prof.err; exit 1; }
S=$(find $R/gpurun_out/prof_purchase -name '*kernel_stats.csv' | head -1)
python3 $R/scripts/gpu_us_per_msg.py $S $R/gpurun_out/purchase_prof.json --out $R/gpurun_out/gpu_us_purchase.json
find $R/gpurun_out/prof_purchase -type f ! -name '*kernel_stats.csv' -delete
