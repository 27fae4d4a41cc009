#!/bin/bash
# round 6, call S: bench.py through the driver's multi-GPU launcher (torch.distributed.run,
# one rank) -- the env-var rendezvous path the N > 1 scaling runs take
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
tail -c 800 $O/bench.json
