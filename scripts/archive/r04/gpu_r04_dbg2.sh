#!/bin/bash
# r04: the broken-answer bench again (20 steps, --profile-cpu), recording non-parsed answers
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export SMSGATE_DEBUG_ANSWERS=$R/gpurun_out/dbg_answers
timeout -k 10 700 python3 -u bench.py --steps 20 --warmup 2 --verbose --profile-cpu /tmp/cprof_dbg --ingest bus \
  --weights-cache /tmp/dbg2 > gpurun_out/dbg2.json 2> gpurun_out/dbg2.err || { tail -20 gpurun_out/dbg2.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/dbg2.json') if l.startswith('{')][-1])
print('value', d['value'], 'routing', d['routing'], 'engine', json.dumps(d.get('engine'))[:600])"
ls gpurun_out/dbg_answers | head; cat gpurun_out/dbg_answers/*.jsonl | head -c 3000
