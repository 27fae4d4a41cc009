#!/bin/bash
# Engine tests + A/B of row compaction x bucket granularity on the headline bench.
set -o pipefail
mkdir -p gpurun_out
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_eng.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_eng.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_eng.log; exit $rc; }
for cfg in "" "--no-compact"; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --verbose $cfg > gpurun_out/ab.log 2>&1 || exit 1
  echo "[$cfg] $(grep metric gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("engine",{}); print(d["value"], e.get("decode_steps"), e.get("decode_row_steps"), e.get("compactions"), e.get("rows_moved"))')"
done
