#!/bin/bash
# r04: where do span answers break in the bench? small span model; A = trained in-run
# (in-memory weights) + quality eval, B = cached weights without eval, C = cached + eval
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
C="python3 -u $R/bench.py --model small --answer-format span --train-steps 1500 --train-batch 64 --train-lr 2e-3 \
  --steps 4 --warmup 1 --quality-floor 0 --ingest bus --weights-cache /tmp/spandbg --verbose"
timeout -k 10 300 $C --eval-n 200 > $R/gpurun_out/dbg_A.json 2> $R/gpurun_out/dbg_A.err || { tail -20 $R/gpurun_out/dbg_A.err; exit 1; }
timeout -k 10 200 $C --eval-n 0 > $R/gpurun_out/dbg_B.json 2> $R/gpurun_out/dbg_B.err || { tail -20 $R/gpurun_out/dbg_B.err; exit 1; }
timeout -k 10 200 $C --eval-n 200 > $R/gpurun_out/dbg_C.json 2> $R/gpurun_out/dbg_C.err || { tail -20 $R/gpurun_out/dbg_C.err; exit 1; }
for x in A B C; do python3 -c "
import json,sys; d=json.loads([l for l in open('$R/gpurun_out/dbg_$x.json') if l.startswith('{')][-1])
print('$x', d['value'], d['routing'], d.get('weights','')[:60], json.dumps(d.get('engine',{}))[:300])"; done
