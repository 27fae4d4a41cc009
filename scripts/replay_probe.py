#!/usr/bin/env python3
"""Host cost of a decode-graph replay: is the launch asynchronous?

For each engine variant (single batch / split halves in one graph / split halves
as two graphs on two streams), replays the 8192-row decode graph N times
back to back and reports host ms per replay (should be ≪ the GPU time if the
launch is asynchronous) and GPU ms per replay (events).
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def probe(eng, B: int, n: int = 10) -> dict:
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(n):
        eng._run_decode(B)
    t_host = (time.perf_counter() - t0) / n
    e1.record()
    torch.cuda.synchronize()
    return {"host_ms": round(t_host * 1000, 3), "gpu_ms": round(e0.elapsed_time(e1) / n, 3)}


def main() -> None:
    from smsgate_amd.parse.backends.local_llm import build_engine

    out = {}
    for name, kw in [("single", dict(split_decode=0)), ("split_one_graph", dict(split_decode=4096, split_graphs=1)),
                     ("split_two_graphs", dict(split_decode=4096, split_graphs=2))]:
        try:
            eng = build_engine("smollm-135m", device="cuda", random_init=True, answer_format="copy", max_slots=8192, steps_per_graph=2,
                               buckets=(4096, 8192), **kw)
        except TypeError as exc:  # option not available in this build
            out[name] = str(exc)
            continue
        eng.done.fill_(0)  # every row "active" so attention does full work
        out[name] = probe(eng, 8192)
        del eng
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
