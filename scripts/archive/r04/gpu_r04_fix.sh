#!/bin/bash
# r04: the done-row NaN fix -- span GPU tests (NaN-memory regression included), then the
# configuration that broke (trained in-process, 20 steps) with the post-phase check
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_span_gpu.py -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/span_pytest3.log 2>&1
rc=$?; grep -E "PASS|FAIL|TEMPLATES|passed|failed|^E " gpurun_out/span_pytest3.log | cut -c1-300 | tail -20
if [ $rc -gt 1 ]; then exit 1; fi
timeout -k 10 700 python3 -u bench.py --steps 20 --warmup 2 --verbose --eval-after \
  > gpurun_out/fix.json 2> gpurun_out/fix.err || { tail -20 gpurun_out/fix.err; exit 1; }
grep "after the timed" gpurun_out/fix.err
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/fix.json') if l.startswith('{')][-1]); e=d['engine']
print('value', d['value'], d['routing'], 'row_steps/msg', round(e['decode_row_steps']/e['completed'],2))
print('cpu', d['cpu']); print('http', d['http_ingest']['value'], d['http_ingest']['routing'], d['http_ingest']['cpu'])
print('quality', json.dumps(d['quality_heldout_formats'])[:300], d['quality_heldout']['reference_cases'])"
