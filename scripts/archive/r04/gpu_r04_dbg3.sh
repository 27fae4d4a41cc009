#!/bin/bash
# r04: which knob breaks span answers in the bench?  A = 20 steps without --profile-cpu (trains);
# B = 8 steps with --profile-cpu; C = 20 steps with --profile-cpu
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
C="python3 -u bench.py --warmup 2 --verbose --ingest bus --weights-cache /tmp/dbg3"
timeout -k 10 700 $C --steps 20 --eval-n 100 > gpurun_out/dbg3_A.json 2> gpurun_out/dbg3_A.err || { tail -20 gpurun_out/dbg3_A.err; exit 1; }
timeout -k 10 200 $C --steps 8 --eval-n 0 --profile-cpu /tmp/cp_B > gpurun_out/dbg3_B.json 2> gpurun_out/dbg3_B.err || { tail -20 gpurun_out/dbg3_B.err; exit 1; }
timeout -k 10 200 $C --steps 20 --eval-n 0 --profile-cpu /tmp/cp_C > gpurun_out/dbg3_C.json 2> gpurun_out/dbg3_C.err || { tail -20 gpurun_out/dbg3_C.err; exit 1; }
for x in A B C; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/dbg3_$x.json') if l.startswith('{')][-1]); e=d['engine']
print('$x', d['value'], d['routing'], 'row_steps/msg', round(e['decode_row_steps']/e['completed'],2), 'prefill_s', e['prefill_s'], 'admit_s', e['admit_s'])"; done
