#!/bin/bash
# round 6, call A: the qa head's confidence / abstention kernel tests, then the seed probe
# of the widened value grammar (4 training samples concurrently on the one GPU)
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_qa_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06a_pytest_qa.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r06a_pytest_qa.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 960 python -u scripts/qa_seeds.py --tag grammar_v1 --out gpurun_out/r06a_qa_seeds.jsonl \
  --log-dir gpurun_out/r06a_seeds > gpurun_out/r06a_seeds.log 2>&1
rc2=$?
echo "seeds rc=$rc2"
tail -3 gpurun_out/r06a_seeds.log
exit $rc2
