#!/bin/bash
# round 6, call O: prefill attention tests (auto = st32 now, st64pf added), then the
# headline bench on that tree
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_qa_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "attn_prefill or qa" > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; fi
timeout -k 10 900 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['http_ingest']['value'], d['cpu']['cpu_us_per_msg'], d['cpu']['node_cores_at_8_gpus'], d['quality_heldout_formats']['exact'], d['quality_heldout_values']['exact'], d['quality_negatives']['false_parsed_rate'])"
