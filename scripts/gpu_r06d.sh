#!/bin/bash
# round 6, call D: the qa decoder's card rules on the GPU (kernel == host), then the
# quality probe of the widened credit grammar: two learning rates x three training
# samples, all six concurrently on the one GPU
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_qa_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06d_pytest_qa.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r06d_pytest_qa.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u scripts/qa_seeds.py --seeds 0,1,2 --workers 2 \
  --variants '[{"tag": "credit_lr1e3", "overrides": {}}, {"tag": "credit_lr5e4", "overrides": {"lr": 0.0005}}]' \
  --out gpurun_out/r06d_qa_seeds.jsonl --log-dir gpurun_out/r06d_seeds > gpurun_out/r06d_seeds.log 2>&1
rc2=$?
echo "seeds rc=$rc2"
tail -4 gpurun_out/r06d_seeds.log
exit $rc2
