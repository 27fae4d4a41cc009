#!/bin/bash
# One iteration of kernel work: GPU tests -> VALU/MFMA counters on gate_up -> microbench -> headline bench.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_gpu.log; exit $rc; }
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc -o p2 -- python $R/scripts/gemm_pmc.py > $R/gpurun_out/pmc/p2.log 2>&1) || exit 1
timeout -k 10 300 python scripts/kbench.py --batch 4096 --ctx 75 > gpurun_out/kbench.json 2> gpurun_out/kbench.err || { tail gpurun_out/kbench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/kbench.json'));print({k:v for k,v in d.items() if 'auto' in k or 'cascade' in k or 'est' in k or 'rope' in k})"
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench.log 2>&1
rc=$?; grep metric gpurun_out/bench.log | cut -c1-150; exit $rc
