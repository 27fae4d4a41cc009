# Round-3 session 2: the two decode halves as one fork/join graph with the second half one
# QKV GEMM behind (split_graphs 1, offset on) vs the default two per-half graphs replayed
# together (no offset), interleaved, three runs per arm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/ab.py --out gpurun_out/r03s2_ab_offset.jsonl --repeats 3 --timeout 500 \
  --arm "g2=" --arm "g1=--split-graphs 1" --common=--verbose > gpurun_out/r03s2_ab_offset.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_offset.log; exit 1; }
tail -4 gpurun_out/r03s2_ab_offset.log
