#!/bin/bash
# speed-of-light table with the verify attention rotating through 8 disjoint KV regions,
# then the measured HBM bytes (FETCH_SIZE / WRITE_SIZE) of every case
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sol_table.py > gpurun_out/r03s3_sol2.json 2> gpurun_out/r03s3_sol2.log && cat gpurun_out/r03s3_sol2.json &&
timeout -k 10 700 bash scripts/gpu_r03_solpmc.sh
