set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/r02_first_bench.log 2>&1
rc=$?; tail -3 gpurun_out/r02_first_bench.log; exit $rc
