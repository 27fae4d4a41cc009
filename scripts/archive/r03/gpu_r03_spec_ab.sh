# Speculative-decoding knobs re-checked on the number-aware tokenizer (shorter answers).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/ab.py --out gpurun_out/r03_ab_spec.jsonl --repeats 2 --timeout 400 --arm "base=" --arm "frac1.5=--spec-frac 1.5" --arm "frac1.0=--spec-frac 1.0" --arm "k8=--spec-k 8" --common "--steps 12 --warmup 2 --eval-n 0 --verbose" > gpurun_out/r03_ab_spec.log 2>&1
rc=$?; tail -6 gpurun_out/r03_ab_spec.log; exit $rc
