# Round-3 session 2: the gate/up kernel under two concurrent decode halves at the new
# default: persistent 256x256 (cfg 20, default) vs one tile per block (cfg 19) vs 128x128
# 8-wave (cfg 13), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/ab.py --out gpurun_out/r03s2_ab_swiglu.jsonl --repeats 2 --timeout 500 \
  --arm "s20=" --arm "s19=--swiglu-cfg 19" --arm "s13=--swiglu-cfg 13" \
  --common=--verbose > gpurun_out/r03s2_ab_swiglu.log 2>&1 || { tail -8 gpurun_out/r03s2_ab_swiglu.log; exit 1; }
tail -4 gpurun_out/r03s2_ab_swiglu.log
