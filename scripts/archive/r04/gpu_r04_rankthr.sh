#!/bin/bash
# r04: which launch mode makes the rank process's busy ROCm runtime thread?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
C="python3 -u bench.py --steps 12 --warmup 2 --verbose --ingest bus --weights-cache /tmp/rkt"
timeout -k 10 600 $C --eval-n 0 > gpurun_out/rt_0.json 2> gpurun_out/rt_0.err || { tail -20 gpurun_out/rt_0.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --no-graphs > gpurun_out/rt_1.json 2> gpurun_out/rt_1.err || { tail -20 gpurun_out/rt_1.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --split-graphs 1 > gpurun_out/rt_2.json 2> gpurun_out/rt_2.err || { tail -20 gpurun_out/rt_2.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --split-decode 0 --split-prefill 0 > gpurun_out/rt_3.json 2> gpurun_out/rt_3.err || { tail -20 gpurun_out/rt_3.err; exit 1; }
for x in 0 1 2 3; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/rt_$x.json') if l.startswith('{')][-1]); c=d['cpu']
print('$x', d['value'], 'broken', d['routing']['broken'], c['cores_busy_per_gpu'], c['cpu_us_per_msg'], c.get('rank_threads_cores', [])[:3])"; done
