#!/bin/bash
# round 6, call F: the fourth training sample (seed 3) of the round-6 recipe (lr 5e-4),
# a lower-lr variant on seeds 0-2, and the bundled small extractor retrained with the
# recipe -- five trainings concurrently on the one GPU
mkdir -p gpurun_out
timeout -k 10 1050 python -u scripts/train_small_asset.py --out gpurun_out/r06f_extractor-small.safetensors \
  > gpurun_out/r06f_small.json 2> gpurun_out/r06f_small.err &
small=$!
timeout -k 10 1050 python -u scripts/qa_seeds.py --workers 2 \
  --variants '[{"tag": "r6_lr5e4", "seeds": [3], "overrides": {}}, {"tag": "r6_lr3e4", "seeds": [0, 1, 2], "overrides": {"lr": 0.0003}}]' \
  --out gpurun_out/r06f_qa_seeds.jsonl --log-dir gpurun_out/r06f_seeds > gpurun_out/r06f_seeds.log 2>&1
rc=$?
wait $small
rc2=$?
echo "seeds rc=$rc small rc=$rc2"
tail -3 gpurun_out/r06f_seeds.log
cat gpurun_out/r06f_small.json
exit $(( rc > rc2 ? rc : rc2 ))
