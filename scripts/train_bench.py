#!/usr/bin/env python3
"""Extractor training throughput (fwd + bwd + AdamW, bf16 autocast) on one GPU.

Times ``--steps`` optimizer steps after ``--warmup`` of the trainer's own loop
(:func:`smsgate_amd.models.train.train_extractor`, single rank: the bucketed
all-reduce is a no-op) and reports answer-tokens/s and sequence-tokens/s.
Under ``torchrun`` every rank trains its own data-parallel shard.

    python scripts/train_bench.py --model smollm-135m --batch 64 --steps 30
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="smollm-135m")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    import torch

    from smsgate_amd.models.train import TrainConfig, train_extractor

    stamps = []

    def log(msg: str) -> None:
        torch.cuda.synchronize()
        stamps.append((time.perf_counter(), msg))

    total = a.warmup + a.steps
    cfg = TrainConfig(model=a.model, steps=total, batch=a.batch, n_examples=4000, log_every=1, warmup=2)
    train_extractor(cfg, device="cuda", log=log)
    steps = [(t, m) for t, m in stamps if m.startswith("step")]
    t0, t1 = steps[a.warmup][0], steps[-1][0]
    dt = (t1 - t0) / (len(steps) - 1 - a.warmup)
    res = {"model": a.model, "batch": a.batch, "ms_per_step": round(dt * 1000, 2),
           "seqs_per_s": round(a.batch / dt, 1), "last": steps[-1][1]}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
