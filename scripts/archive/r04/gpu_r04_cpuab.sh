#!/bin/bash
# r04: host CPU knobs, span answers, weights trained once then reused: default vs one torch
# thread in the rank process vs also one tokenizer thread per parser process
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
C="python3 -u bench.py --steps 20 --warmup 2 --verbose --ingest bus --weights-cache /tmp/cpuab"
timeout -k 10 600 $C --eval-n 100 > gpurun_out/cpuab_0.json 2> gpurun_out/cpuab_0.err || { tail -20 gpurun_out/cpuab_0.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 --rank-threads 1 > gpurun_out/cpuab_1.json 2> gpurun_out/cpuab_1.err || { tail -20 gpurun_out/cpuab_1.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 --rank-threads 1 --worker-threads 1 > gpurun_out/cpuab_2.json 2> gpurun_out/cpuab_2.err || { tail -20 gpurun_out/cpuab_2.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 > gpurun_out/cpuab_3.json 2> gpurun_out/cpuab_3.err || { tail -20 gpurun_out/cpuab_3.err; exit 1; }
for x in 0 1 2 3; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/cpuab_$x.json') if l.startswith('{')][-1]); c=d['cpu']
print('$x', d['value'], 'broken', d['routing']['broken'], c['cores_busy_per_gpu'], c['cpu_us_per_msg'], c['node_cores_at_8_gpus'])"; done
