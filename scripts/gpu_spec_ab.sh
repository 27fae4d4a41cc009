#!/bin/bash
# Speculative decoding A/B on the headline bench (weights trained once, cached), then latency.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 0 4 0 4; do
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --verbose --eval-n 0 --spec-k $k > gpurun_out/spec_ab_k$k.log 2>&1
  rc=$?; tail -1 gpurun_out/spec_ab_k$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('engine',{}); print('k=$k', d['value'], d['routing'], {x: e.get(x) for x in ('spec_tokens_per_row_step','decode_steps','decode_row_steps','prefill_tokens')})"; [ $rc -eq 0 ] || exit $rc
done
