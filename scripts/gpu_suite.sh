#!/bin/bash
# One GPU-box driver for the recurring stages (replaces round 1's gpu_*.sh one-offs).
#
#   bash scripts/gpu_suite.sh tests smoke bench profile latency
#
# Stages (run in the order given, each under its own time limit; the first
# failure ends the call — nothing more touches the GPU after it):
#   tests     GPU test suite in one process        -> gpurun_out/pytest_gpu.log
#   smoke     __graft_entry__.smoke()               -> gpurun_out/smoke.log
#   bench     bench.py with defaults (--verbose)    -> gpurun_out/bench.log
#   profile   rocprofv3 kernel stats of bench.py    -> gpurun_out/prof/
#   latency   Poisson serving latency, trained weights, spec on/off -> gpurun_out/latency_spec{0,4}.json
#   curve     extractor training curve (held-out accuracy) -> gpurun_out/curve.log
#   worst     bench.py with random-init weights (every answer runs to the field caps) -> gpurun_out/bench_random.log
#   ktests    GPU tests selected by PYTEST_K (pytest -k) -> gpurun_out/ktests.log
#   tune      scripts/gemm_tune.py $TUNE_ARGS        -> gpurun_out/gemm_tune.json
# Extra bench.py arguments can be passed in BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
for stage in "$@"; do
  case $stage in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -3 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
      rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200 ;;
    bench)
      timeout -k 10 900 python -u bench.py --verbose $BENCH_ARGS > gpurun_out/bench.log 2>&1
      rc=$?; tail -1 gpurun_out/bench.log | cut -c1-600 ;;
    profile)
      # first run trains + caches the weights, the profiled run reuses them
      timeout -k 10 700 python -u bench.py --steps 2 --warmup 1 --eval-n 0 $BENCH_ARGS > gpurun_out/prof_warm.log 2>&1 || { rc=$?; tail -3 gpurun_out/prof_warm.log; exit $rc; }
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 $BENCH_ARGS > $R/gpurun_out/prof.log 2>&1)
      rc=$?; tail -1 gpurun_out/prof.log | cut -c1-160
      # the trace itself is too big to copy back: keep a (kernel, grid) histogram of it
      [ $rc -eq 0 ] && python scripts/prof_summary.py gpurun_out/prof
      find gpurun_out/prof -name "*kernel_trace.csv" -delete ;;
    ktests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ktests.log 2>&1
      rc=$?; tail -3 gpurun_out/ktests.log ;;
    tune)
      timeout -k 10 600 python -u scripts/gemm_tune.py $TUNE_ARGS > gpurun_out/gemm_tune.json 2> gpurun_out/gemm_tune.err
      rc=$?; tail -c 600 gpurun_out/gemm_tune.json ;;
    latency)
      rc=0
      for k in 0 4; do
        timeout -k 10 400 python -u scripts/latency_bench.py --weights train --spec-k $k --rates 1000,2000,6000,10000,14000 --seconds 4 --out gpurun_out/latency_spec$k.json > gpurun_out/latency_spec$k.log 2>&1
        rc=$?; grep offered gpurun_out/latency_spec$k.log | cut -c1-150; [ $rc -eq 0 ] || break
      done ;;
    worst)
      timeout -k 10 600 python -u bench.py --weights random --eval-n 0 $BENCH_ARGS > gpurun_out/bench_random.log 2>&1
      rc=$?; tail -1 gpurun_out/bench_random.log | cut -c1-400 ;;
    curve)
      timeout -k 10 900 python -u scripts/train_curve.py $CURVE_ARGS > gpurun_out/curve.log 2>&1
      rc=$?; grep '"step"' gpurun_out/curve.log | cut -c1-300 ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || { echo "stage $stage failed (rc $rc)"; exit $rc; }
done
