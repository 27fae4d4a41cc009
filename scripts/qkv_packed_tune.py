#!/usr/bin/env python3
"""QKV+RoPE GEMM tile configs at the qa engine's real layout: packed sequences (positions
0.. per sequence, one KV slot each, ~53 rows a message), so V^T blocks are whole -- the
random positions of scripts/gemm_tune.py send every V^T write down the per-element path
and overstate the V part.  One JSON line: microseconds per config (graph replay median)."""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from smsgate_amd import ops  # noqa: E402
from scripts.gemm_tune import graph_time  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=110592)
    p.add_argument("--cfgs", default="28,39,40,41")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--inner", type=int, default=5)
    a = p.parse_args()
    dev, nh, nkv, D, K, Lmax, p0 = "cuda", 9, 3, 64, 576, 192, 20
    g = torch.Generator(device="cpu").manual_seed(5)
    lens = []
    while sum(lens) < a.rows:
        lens.append(int(torch.randint(40, 67, (1,), generator=g)))
    lens[-1] -= sum(lens) - a.rows
    S = len(lens)
    M = a.rows
    pos = torch.cat([torch.arange(n) for n in lens]).to(torch.int32).to(dev)
    slot = torch.repeat_interleave(torch.arange(S), torch.tensor(lens)).to(torch.int32).to(dev)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    w = (torch.randn((nh + 2 * nkv) * D, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    ss = ops.ss_buffer(M, dev)
    ss[:6] = x.float().pow(2).view(M, 6, 96).sum(-1).t()
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, dev)
    kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=dev)
    vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=dev)
    q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=dev)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    best = {c: math.inf for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            best[c] = min(best[c], graph_time(
                lambda: ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, cfg=c, ss_in=ss),
                a.iters, a.inner))
    print(json.dumps({"rows": M, "seqs": S, "us": {c: round(t, 2) for c, t in best.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
