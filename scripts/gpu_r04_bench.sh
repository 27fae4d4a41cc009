#!/bin/bash
# r04: the headline bench in one answer format (FMT=copy|span) with CPU profiles, then a
# rocprofv3 kernel-stats run of the serving kernels only (weights from the first run's
# cache, no quality evaluation, one ingest phase) -> GPU us per LLM-routed message
set -o pipefail
FMT=${FMT:-span}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 840 python3 -u $R/bench.py --answer-format $FMT --steps 20 --warmup 2 --verbose \
  --profile-cpu $R/gpurun_out/cprof_$FMT > $R/gpurun_out/bench_$FMT.json 2> $R/gpurun_out/bench_$FMT.err \
  || { tail -20 $R/gpurun_out/bench_$FMT.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$R/gpurun_out/bench_$FMT.json') if l.startswith('{')][-1])
print('value', d['value'], 'routing', d['routing'], 'cpu', d.get('cpu'))
print('quality', json.dumps(d.get('quality_heldout_formats'))[:400], d.get('quality_heldout', {}).get('reference_cases'))
print('http', json.dumps(d.get('http_ingest'))[:500])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$FMT -o run -- python3 $R/bench.py \
  --answer-format $FMT --steps 10 --warmup 2 --eval-n 0 --quality-floor 0 --ingest bus \
  > $R/gpurun_out/bench_${FMT}_prof.json 2> $R/gpurun_out/bench_${FMT}_prof.err \
  || { tail -20 $R/gpurun_out/bench_${FMT}_prof.err; exit 1; }
S=$(find $R/gpurun_out/prof_$FMT -name '*kernel_stats.csv' -o -name '*.db' | sort | head -1)
python3 $R/scripts/gpu_us_per_msg.py $S $R/gpurun_out/bench_${FMT}_prof.json --out $R/gpurun_out/gpu_us_$FMT.json
# keep what comes back under gpurun's 64 MiB: the kernel stats, not the per-dispatch traces
find $R/gpurun_out/prof_$FMT -type f ! -name '*kernel_stats.csv' -delete
if [ "$FMT" = "copy" ]; then  # the verify-attention SOL row at the bench's max_q = 7
  cd $R && timeout -k 10 240 python3 -u scripts/sol_table.py > gpurun_out/r04_sol_maxq7.json 2> gpurun_out/r04_sol.log \
    || { tail -5 gpurun_out/r04_sol.log; exit 1; }
fi
