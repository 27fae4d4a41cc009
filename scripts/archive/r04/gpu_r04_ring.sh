#!/bin/bash
# r04: the 32-slot staging ring -- engine / span GPU tests, then the default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_span_gpu.py tests/test_engine_gpu.py -q --timeout 280 \
  --timeout-method thread > gpurun_out/ring_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/ring_pytest.log; if [ $rc -ne 0 ]; then exit 1; fi
bash scripts/gpu_r04_final.sh && python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/final.json') if l.startswith('{')][-1]); e=d['engine']
print('gpu_idle', e['gpu_idle_s'], 'admit_s', e['admit_s'], 'prefill_s', e['prefill_s'], d['cpu'].get('rank_threads_cores', [])[:2])"
