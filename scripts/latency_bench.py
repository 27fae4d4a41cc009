#!/usr/bin/env python3
"""Serving latency of the extraction engine under a paced (Poisson) arrival stream.

For each offered load R (msgs/s) the host submits pre-tokenised SMS whose
arrival time has passed before every engine step, and records submit → answer
latency per message.  Reports achieved throughput and p50/p95/p99 latency —
the serving-side view of the headline throughput number (the reference's
``sms_parser_processing_seconds`` histogram measured one Gemini round trip per
message).  The qa engine (default) answers in one forward whatever the weights; the
span / copy engines' random-init answers decode the schema's maximum tokens (their
worst case).

    python scripts/latency_bench.py --rates 2000,8000,14000 --seconds 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def run_rate(eng, ids, rate: float, seconds: float, seed: int) -> dict:
    rng = np.random.default_rng(seed)
    n = int(rate * seconds)
    arrivals = np.cumsum(rng.exponential(1.0 / rate, n))
    t_sub = np.zeros(n)
    t_done = np.full(n, np.nan)
    nxt = 0
    t0 = time.perf_counter()
    while nxt < n or eng.busy():
        now = time.perf_counter() - t0
        j = nxt
        while j < n and arrivals[j] <= now:
            j += 1
        if j > nxt:
            eng.submit_ids([(k, ids[k % len(ids)]) for k in range(nxt, j)])
            t_sub[nxt:j] = now
            nxt = j
        if not eng.busy():
            time.sleep(min(0.0005, max(0.0, arrivals[nxt] - now)) if nxt < n else 0)
            continue
        for k, _ in eng.step(raw=True):
            t_done[k] = time.perf_counter() - t0
    wall = time.perf_counter() - t0
    lat = (t_done - t_sub) * 1000.0
    lat = lat[~np.isnan(lat)]
    return {"offered_msgs_per_s": rate, "msgs": int(n), "achieved_msgs_per_s": round(n / wall, 1),
            "p50_ms": round(float(np.percentile(lat, 50)), 1), "p95_ms": round(float(np.percentile(lat, 95)), 1),
            "p99_ms": round(float(np.percentile(lat, 99)), 1), "max_ms": round(float(lat.max()), 1)}


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--rates", default="2000,8000,14000")
    p.add_argument("--seconds", type=float, default=6.0)
    p.add_argument("--max-slots", type=int, default=8192)
    p.add_argument("--out", default=None)
    p.add_argument("--attn-small-rows", type=int, default=None,
                   help="decode buckets up to N rows use --attn-small (default: the engine's)")
    p.add_argument("--attn-small", default="split2")
    p.add_argument("--gemm-small-m", type=int, default=None, help="ops.GEMM_SMALL_M (32-row GEMM tiles up to M)")
    p.add_argument("--admit-min-batch", type=int, default=None,
                   help="EngineConfig.admit_min_batch (0 = off; default: the engine's)")
    p.add_argument("--admit-max-wait-ms", type=float, default=None)
    p.add_argument("--prefill-key-split", type=int, default=None, choices=[1, 2])
    p.add_argument("--weights", default="random",
                   help="random | train (bench.py's in-run training, reusing its weights cache) | checkpoint path")
    p.add_argument("--spec-k", type=int, default=0, help="speculative decoding drafts per row (0 = off)")
    p.add_argument("--answer-format", default="qa", choices=["qa", "span", "copy"],
                   help="qa: the one-forward engine (serving/qa_engine.py, the default extractor); span / copy: the "
                        "autoregressive engine of rounds 3-4")
    p.add_argument("--traffic", default="formats", help="utils/synth.py TRAFFIC preset of the offered SMS")
    p.add_argument("--qa-max-tokens", type=int, default=None)
    p.add_argument("--qa-min-tokens", type=int, default=None)
    p.add_argument("--profile", default=None, choices=["throughput", "latency", "latency_r2"],
                   help="engine configuration of serving/profiles.py (what engine-server --profile serves); "
                        "--max-slots / --spec-k are then ignored")
    a = p.parse_args()
    import torch

    from smsgate_amd import ops
    from smsgate_amd.parse.backends.local_llm import build_engine
    from smsgate_amd.parse.text import normalize_body
    
    if a.gemm_small_m is not None:
        ops.GEMM_SMALL_M = a.gemm_small_m
    kw = {} if a.attn_small_rows is None else dict(decode_attn_small_rows=a.attn_small_rows,
                                                   decode_attn_small=a.attn_small)
    if a.admit_min_batch is not None:
        kw["admit_min_batch"] = a.admit_min_batch
    if a.prefill_key_split is not None:
        kw["prefill_key_split"] = a.prefill_key_split
    if a.admit_max_wait_ms is not None:
        kw["admit_max_wait_s"] = a.admit_max_wait_ms / 1000.0
    if a.qa_max_tokens is not None:
        kw["qa_max_tokens"] = a.qa_max_tokens
    if a.qa_min_tokens is not None:
        kw["qa_min_tokens"] = a.qa_min_tokens
    weights = None
    if a.weights != "random":
        import bench

        bargs = bench._args(["--weights", a.weights, "--answer-format", a.answer_format])
        weights, _ = bench.acquire_weights(bargs, "cuda:0", 0, 1)
    if a.profile:
        from smsgate_amd.serving.profiles import profile_kwargs

        ekw = dict(profile_kwargs(a.profile), **kw)
    else:
        ekw = dict(max_slots=a.max_slots, steps_per_graph=2, buckets=(64, 128, 256, 512, 1024, 2048, 4096, 8192),
                   spec_k=a.spec_k, **kw)
    eng = build_engine("smollm-135m", device="cuda", random_init=weights is None, weights=weights,
                       answer_format=a.answer_format, **ekw)
    a.spec_k = eng.cfg.spec_k
    arm = {"profile": a.profile, "answer_format": a.answer_format, "traffic": a.traffic,
           "weights": a.weights, "engine": type(eng).__name__}
    if a.answer_format == "qa":
        arm.update(qa_max_tokens=eng.cfg.qa_max_tokens, qa_min_tokens=eng.cfg.qa_min_tokens, max_slots=eng.cfg.max_slots)
    else:
        arm.update(attn_small_rows=eng.cfg.decode_attn_small_rows, attn_small=eng.cfg.decode_attn_small,
                   gemm_small_m=ops.GEMM_SMALL_M, admit_min_batch=eng.cfg.admit_min_batch,
                   admit_max_wait_ms=eng.cfg.admit_max_wait_s * 1000.0, prefill_key_split=eng.cfg.prefill_key_split,
                   spec_k=a.spec_k)
    from smsgate_amd.utils.synth import generate_traffic

    bodies = [normalize_body(s.body) for s in generate_traffic(20000, seed=5, traffic=a.traffic)]
    ids = eng.tok.message_ids(bodies, eng.cfg.max_body_tokens)
    run_rate(eng, ids, 2000.0, 1.0, seed=0)  # warm-up
    torch.cuda.synchronize()
    res = [dict(run_rate(eng, ids, float(r), a.seconds, seed=i + 1), **arm) for i, r in enumerate(a.rates.split(","))]
    for r in res:
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
