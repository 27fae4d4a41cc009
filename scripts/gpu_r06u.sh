#!/bin/bash
# round 6, call U: the whole GPU suite, smoke() and the headline bench after the 33-broker layout
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
  || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
echo "smoke ok"; tail -2 $O/smoke.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['http_ingest']['value'], d['cpu']['cpu_us_per_msg'], d['cpu']['node_cores_at_8_gpus'], d['quality_heldout_formats']['exact'], d['quality_heldout_values']['exact'], d['quality_negatives']['false_parsed_rate'])"
