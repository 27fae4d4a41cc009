#!/usr/bin/env python3
"""Where a training step's time goes (the bench trains the flagship in-run, untimed):
ms per step of the bench recipe (135M, batch 128, bf16 autocast, fused AdamW, EMA),
the GPU kernel time inside a step (torch.profiler), and the kernel count -- a step
that launches thousands of small kernels is launch-bound, not FLOP-bound."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--format", default="qa")
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--fused", default="1,0", help="TrainConfig.fused values to measure (A/B)")
    a = p.parse_args()
    import torch

    from smsgate_amd.models.train import TrainConfig, answer_fsm, make_examples, train_extractor
    from smsgate_amd.models.tokenizer import load_tokenizer

    tok = load_tokenizer()
    data = make_examples(tok, answer_fsm(tok, a.format), 8192, seed=1, negatives=0.12)
    for fused in (bool(int(x)) for x in a.fused.split(",")):
        times = []

        def log(s):
            times.append((time.perf_counter(), s))

        tc = TrainConfig(steps=a.steps, batch=a.batch, n_examples=len(data), log_every=1, answer_format=a.format,
                         warmup=5, fused=fused)
        train_extractor(tc, device="cuda", data=data, log=log)
        stamps = [t for t, s in times if s.startswith("step")]
        per = (stamps[-1] - stamps[10]) / (len(stamps) - 11) * 1e3
        # one profiled step range (kernel count and GPU time)
        from torch.profiler import ProfilerActivity, profile

        tc2 = TrainConfig(steps=6, batch=a.batch, n_examples=len(data), log_every=0, answer_format=a.format,
                          warmup=2, fused=fused)
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            train_extractor(tc2, device="cuda", data=data, log=lambda s: None)
            torch.cuda.synchronize()
        kev = [e for e in prof.key_averages() if getattr(e, "self_device_time_total", 0) > 0]
        kern = sum(e.count for e in kev)
        gpu_us = sum(e.self_device_time_total for e in kev)
        top = sorted(kev, key=lambda e: -e.self_device_time_total)[:12]
        print(json.dumps({"format": a.format, "batch": a.batch, "fused": fused, "ms_per_step": round(per, 2),
                          "kernels_per_step": round(kern / 6, 1), "gpu_ms_per_step": round(gpu_us / 6 / 1e3, 2),
                          "top": [[e.key[:60], round(e.self_device_time_total / 6 / 1e3, 3), e.count // 6]
                                  for e in top]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
