#!/bin/bash
# r04: trained in-process + 20 steps breaks span answers; is the engine state corrupted
# (quality / weights after the phases), or the serving path?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export SMSGATE_DEBUG_ANSWERS=$R/gpurun_out/dbg4_answers
timeout -k 10 700 python3 -u bench.py --steps 20 --warmup 2 --verbose --ingest bus --eval-n 100 --eval-after \
  > gpurun_out/dbg4.json 2> gpurun_out/dbg4.err || { tail -20 gpurun_out/dbg4.err; exit 1; }
grep "after the timed" gpurun_out/dbg4.err
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/dbg4.json') if l.startswith('{')][-1]); e=d['engine']
print('value', d['value'], d['routing'], 'row_steps/msg', round(e['decode_row_steps']/e['completed'],2))"
