#!/bin/bash
# r04: the 135M span bench answered ~86 % of the timed messages card-less while its
# in-process quality eval (same engine) was 97 % exact, and a rocprofv3 run (kernels
# serialised) routed correctly.  1 = default (trains, evals); 2 = no split decode /
# prefill (one stream); 3 = default again without the eval; 4 = no templates
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
C="python3 -u $R/bench.py --answer-format span --steps 8 --warmup 1 --ingest bus --verbose --weights-cache /tmp/race"
timeout -k 10 600 $C --eval-n 100 > $R/gpurun_out/race_1.json 2> $R/gpurun_out/race_1.err || { tail -20 $R/gpurun_out/race_1.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 --split-decode 0 --split-prefill 0 > $R/gpurun_out/race_2.json 2> $R/gpurun_out/race_2.err || { tail -20 $R/gpurun_out/race_2.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 > $R/gpurun_out/race_3.json 2> $R/gpurun_out/race_3.err || { tail -20 $R/gpurun_out/race_3.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 --template-slots 0 > $R/gpurun_out/race_4.json 2> $R/gpurun_out/race_4.err || { tail -20 $R/gpurun_out/race_4.err; exit 1; }
for x in 1 2 3 4; do python3 -c "
import json,sys; d=json.loads([l for l in open('$R/gpurun_out/race_$x.json') if l.startswith('{')][-1])
e=d.get('engine',{})
print('$x', d['value'], d['routing'], 'row_steps/msg', round(e.get('decode_row_steps',0)/max(1,e.get('completed',1)),2), 'steps', e.get('decode_steps'))"; done
