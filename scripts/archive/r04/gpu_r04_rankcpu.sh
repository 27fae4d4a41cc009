#!/bin/bash
# r04: what burns the rank process's second core (a native thread at ~0.94 core)?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
C="python3 -u bench.py --steps 20 --warmup 2 --verbose --ingest bus --weights-cache /tmp/rankcpu"
timeout -k 10 600 $C --eval-n 50 > gpurun_out/rk_0.json 2> gpurun_out/rk_0.err || { tail -20 gpurun_out/rk_0.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 --no-measure-idle > gpurun_out/rk_1.json 2> gpurun_out/rk_1.err || { tail -20 gpurun_out/rk_1.err; exit 1; }
ROC_ACTIVE_WAIT_TIMEOUT=0 timeout -k 10 200 $C --eval-n 0 > gpurun_out/rk_2.json 2> gpurun_out/rk_2.err || { tail -20 gpurun_out/rk_2.err; exit 1; }
HSA_ENABLE_INTERRUPT=1 timeout -k 10 200 $C --eval-n 0 --no-measure-idle > gpurun_out/rk_3.json 2> gpurun_out/rk_3.err || { tail -20 gpurun_out/rk_3.err; exit 1; }
for x in 0 1 2 3; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/rk_$x.json') if l.startswith('{')][-1]); c=d['cpu']
print('$x', d['value'], 'broken', d['routing']['broken'], c['cores_busy_per_gpu'], c['cpu_us_per_msg'], c.get('rank_threads_cores', [])[:3])"; done
