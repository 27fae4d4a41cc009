#!/usr/bin/env python3
"""Prefill attention microbench at the engine's shapes: per-head, GQA-shared and
multi-tile and transposed register kernels (one JSON line per batch size).

    python scripts/prefill_bench.py [--nseq 150,300,800] [--out gpurun_out/prefill_bench.jsonl]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from smsgate_amd import ops  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--nseq", default="150,300,800")
    p.add_argument("--lens", default="40,70", help="prompt length range (tokens)")
    p.add_argument("--nh", type=int, default=9)
    p.add_argument("--nkv", type=int, default=3)
    p.add_argument("--P0", type=int, default=20)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--out", default=None)
    p.add_argument("--impls", default="per_head,gqa,gqa_ks2,multi,st,st32,st64,st32pf,stpf,st64pf")
    a = p.parse_args()
    lines = [run(a, int(n)) for n in a.nseq.split(",")]
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write("".join(json.dumps(r) + "\n" for r in lines))


def run(a, nseq: int) -> dict:
    dev = "cuda"
    a.nseq = nseq
    lo, hi = (int(x) for x in a.lens.split(","))
    g = torch.Generator(device="cpu").manual_seed(0)
    lens = torch.randint(lo, hi, (a.nseq,), generator=g).tolist()
    D, Lmax = 64, 192
    S = a.nseq
    T = sum(lens)
    P0pad = (a.P0 + 31) // 32 * 32
    q = (torch.randn(T, a.nh, D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    kc = (torch.randn(S, a.nkv, Lmax, D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    vt = ops.rows_to_vt((torch.randn(S, a.nkv, Lmax, D, generator=g) * 0.5).to(torch.bfloat16).to(dev))
    pk = (torch.randn(a.nkv, P0pad, D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    pvt = ops.rows_to_vt((torch.randn(a.nkv, P0pad, D, generator=g) * 0.5).to(torch.bfloat16).to(dev))
    cu = torch.tensor([0] + torch.cumsum(torch.tensor(lens), 0).tolist(), dtype=torch.int32, device=dev)
    qs = torch.zeros(a.nseq, dtype=torch.int32, device=dev)
    sl = torch.arange(a.nseq, dtype=torch.int32, device=dev)
    scale = 1 / math.sqrt(D)
    res = {"nseq": a.nseq, "tokens": T, "nh": a.nh, "nkv": a.nkv, "P0": a.P0}
    outs = {}
    for impl in a.impls.split(","):
        ops.set_prefill_impl("gqa" if impl.startswith("gqa") else impl)
        ops.set_prefill_split(2 if impl == "gqa_ks2" else 1)
        out = torch.empty(T, a.nh * D, dtype=torch.bfloat16, device=dev)
        for _ in range(3):
            ops.attn_prefill(q, cu, qs, sl, max(lens), kc, vt, pk, pvt, a.P0, out, scale)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.attn_prefill(q, cu, qs, sl, max(lens), kc, vt, pk, pvt, a.P0, out, scale)
        e1.record()
        torch.cuda.synchronize()
        res[f"{impl}_us"] = round(e0.elapsed_time(e1) / a.iters * 1000, 2)
        outs[impl] = out.float()
    ops.set_prefill_impl("auto")
    ops.set_prefill_split(1)
    ref = "per_head" if "per_head" in outs else next(iter(outs))
    for impl in outs:
        res[f"max_abs_diff_{impl}"] = float((outs[impl] - outs[ref]).abs().max())
        res[f"speedup_{impl}_vs_{ref}"] = round(res[f"{ref}_us"] / res[f"{impl}_us"], 3)
    for a_, b_ in (("st32pf", "st32"), ("stpf", "st"), ("st64pf", "st64")):
        if a_ in outs and b_ in outs:
            res[f"{a_}_bitwise_{b_}"] = bool(torch.equal(outs[a_], outs[b_]))
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
