#!/bin/bash
# r04: engine size / graph depth with span answers (weights trained once, reused)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
C="python3 -u bench.py --steps 20 --warmup 2 --verbose --ingest bus --weights-cache /tmp/slots"
timeout -k 10 600 $C --eval-n 50 > gpurun_out/sl_0.json 2> gpurun_out/sl_0.err || { tail -20 gpurun_out/sl_0.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --max-slots 16384 > gpurun_out/sl_1.json 2> gpurun_out/sl_1.err || { tail -20 gpurun_out/sl_1.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --steps-per-graph 4 > gpurun_out/sl_2.json 2> gpurun_out/sl_2.err || { tail -20 gpurun_out/sl_2.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 > gpurun_out/sl_3.json 2> gpurun_out/sl_3.err || { tail -20 gpurun_out/sl_3.err; exit 1; }
timeout -k 10 240 $C --eval-n 0 --max-slots 16384 > gpurun_out/sl_4.json 2> gpurun_out/sl_4.err || { tail -20 gpurun_out/sl_4.err; exit 1; }
for x in 0 1 2 3 4; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/sl_$x.json') if l.startswith('{')][-1]); e=d['engine']
print('$x', d['value'], 'broken', d['routing']['broken'], 'gpu_idle', e['gpu_idle_s'], 'cpu', d['cpu']['cpu_us_per_msg'])"; done
