#!/bin/bash
# speed-of-light table, verify attention with the bench's max_q (two-column-block kernel)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sol_table.py > gpurun_out/r03s3_sol3.json 2> gpurun_out/r03s3_sol3.log && cat gpurun_out/r03s3_sol3.json
