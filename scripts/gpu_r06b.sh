#!/bin/bash
# round 6, call B: (1) one training sample of the widened grammar with every scored
# item's raw head scores dumped (offline decode / confidence study) and, concurrently,
# the bundled small extractor trained with the flagship recipe; (2) the headline bench
# on this tree (native parse path).
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/qa_diag.py --seed 0 --out gpurun_out/r06b_diag_seed0.npz > gpurun_out/r06b_diag.log 2>&1 &
p1=$!
timeout -k 10 600 python -u scripts/train_small_asset.py --out gpurun_out/r06b_extractor-small.safetensors \
  > gpurun_out/r06b_small.json 2> gpurun_out/r06b_small.err &
p2=$!
wait $p1; rc1=$?
wait $p2; rc2=$?
echo "diag rc=$rc1 small rc=$rc2"
tail -2 gpurun_out/r06b_diag.log; cat gpurun_out/r06b_small.json
if [ $rc1 -gt 1 ] && [ $rc1 -ne 124 ]; then exit $rc1; fi
if [ $rc2 -gt 1 ] && [ $rc2 -ne 124 ]; then exit $rc2; fi
timeout -k 10 720 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err
rc3=$?
echo "bench rc=$rc3"
tail -c 1500 gpurun_out/r06b_bench.json
exit $rc3
