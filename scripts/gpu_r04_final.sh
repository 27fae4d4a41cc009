#!/bin/bash
# r04: the driver's bench command on the committed defaults (span answers, 4000 training steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 2 --verbose --weights-cache /tmp/fresh_$$ > gpurun_out/final.json 2> gpurun_out/final.err \
  || { tail -20 gpurun_out/final.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/final.json') if l.startswith('{')][-1])
print('value', d['value'], 'train_s', d.get('train_s'), d['routing'])
print('cpu', d['cpu']['cores_busy_per_gpu'], d['cpu']['cpu_us_per_msg'], d['cpu']['node_cores_at_8_gpus'])
print('http', d['http_ingest']['value'], d['http_ingest']['routing'], d['http_ingest']['cpu']['cpu_us_per_msg'])
print('quality', json.dumps(d['quality_heldout_formats'])[:400], d['quality_heldout']['reference_cases'], d['quality_heldout']['legacy_mix']['exact'], d['quality_train_formats']['exact'])"
