#!/bin/bash
# GEMM tile-size threshold under nano-batch overlap.
set -o pipefail
mkdir -p gpurun_out
for mt in 480 240 960 480 240; do
  SMSGATE_GEMM_MIN_TILES=$mt timeout -k 10 300 python bench.py --steps 4 --warmup 1 > gpurun_out/ab_tiles.log 2>&1 || { tail -5 gpurun_out/ab_tiles.log; exit 1; }
  echo "[min_tiles=$mt] $(grep metric gpurun_out/ab_tiles.log | cut -c1-100)" | tee -a gpurun_out/ab_tiles_summary.txt
done
