#!/bin/bash
# speed-of-light table of the hot kernels, then counter passes of the o-proj residual GEMM
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sol_table.py > gpurun_out/r03s3_sol.json 2> gpurun_out/r03s3_sol.log && cat gpurun_out/r03s3_sol.json &&
B=9216 EPI=resid K=576 CFGS=21 timeout -k 10 600 bash scripts/pmc_gemm.sh
