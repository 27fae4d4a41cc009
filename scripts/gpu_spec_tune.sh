set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_spec_gpu.py tests/test_golden_llm_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_spec.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_spec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u scripts/ab.py --out gpurun_out/ab_spec_tune.jsonl --repeats 1 --common "--steps 10 --warmup 2 --eval-n 0" \
  --arm "k4f2=--spec-k 4 --spec-frac 2.0" --arm "k4f15=--spec-k 4 --spec-frac 1.5" --arm "k6f2=--spec-k 6 --spec-frac 2.0" --arm "k3f15=--spec-k 3 --spec-frac 1.5" --arm "k4f2b=--spec-k 4 --spec-frac 2.0"
