#!/usr/bin/env python3
"""Which CPU op launches the training step's host-to-device copies (the step waits on
them: scripts/train_step_profile.py counts 63 per step)."""
from __future__ import annotations

import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from torch.profiler import ProfilerActivity, profile

    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import TrainConfig, answer_fsm, make_examples, train_extractor

    tok = load_tokenizer()
    data = make_examples(tok, answer_fsm(tok, "qa"), 2048, seed=1, negatives=0.12)
    tc = TrainConfig(steps=4, batch=128, n_examples=len(data), log_every=0, answer_format="qa", warmup=2)
    train_extractor(tc, device="cuda", data=data, log=lambda s: None)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        train_extractor(tc, device="cuda", data=data, log=lambda s: None)
        torch.cuda.synchronize()
    by_op, stacks = collections.Counter(), {}
    parents = collections.Counter()
    for e in prof.events():
        for k in getattr(e, "kernels", []) or []:
            if "HtoD" in k.name:
                key = f"{e.name} {e.input_shapes}"
                by_op[key] += 1
                chain, p = [], e.cpu_parent
                while p is not None and len(chain) < 8:
                    chain.append(p.name)
                    p = p.cpu_parent
                parents[" <- ".join(chain)] += 1
                if key not in stacks:
                    stacks[key] = [str(f) for f in (e.stack or [])][:12]
    print(json.dumps({"htod_by_cpu_op": by_op.most_common(20), "parents": parents.most_common(20), "stacks": stacks},
                     indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
