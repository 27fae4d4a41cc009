#!/usr/bin/env python3
"""Rasterisation group (sg_gemm_set_group_m: M-tiles that walk N together) at the qa
engine's GEMM shapes, interleaved rounds, graph-timed like scripts/gemm_tune.py.  The
default 8 was chosen at round 2's 9 k-row decode shapes."""
from __future__ import annotations

import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd import ops  # noqa: E402
from scripts.gemm_tune import graph_time  # noqa: E402


def main() -> int:
    dev, bf16 = "cuda", torch.bfloat16
    H, I, nh, nkv, D, S = 576, 1536, 9, 3, 64, 8192
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*shape):
        return (torch.randn(*shape, generator=g) * 0.05).to(bf16).to(dev)

    M = int(sys.argv[1]) if len(sys.argv) > 1 else 110592
    x, h, resid = bf(M, H), bf(M, I), bf(M, H)
    w_gu, w_down, w_o, w_qkv = bf(2 * I, H), bf(H, I), bf(H, H), bf((nh + 2 * nkv) * D, H)
    out_gu = torch.empty(M, I, dtype=bf16, device=dev)
    ss = ops.ss_buffer(M, dev)
    ss[:6] = torch.rand(6, M, device=dev)
    sso = ops.ss_buffer(M, dev)
    r = torch.arange(M, dtype=torch.int32)
    pos, slot = (r % 50).to(dev), ((r // 50) % S).to(dev)
    cs = ops.rope_table(1024, D, 1e5, device=dev)
    kc = torch.zeros(S, nkv, 160, D, dtype=bf16, device=dev)
    vt = torch.zeros(*ops.vt_shape(S, nkv, D, 160), dtype=bf16, device=dev)
    q = torch.empty(M, nh, D, dtype=bf16, device=dev)
    cases = {
        "gate_up_cfg20": lambda: ops.gemm(x, w_gu, epi="swiglu", norm_eps=1e-5, out=out_gu, cfg=20, ss_in=ss),
        "down_cfg28": lambda: ops.gemm(h, w_down, epi="resid", resid=resid, cfg=28, ss_out=sso),
        "o_cfg28": lambda: ops.gemm(x, w_o, epi="resid", resid=resid, cfg=28, ss_out=sso),
        "qkv_cfg28": lambda: ops.gemm_qkv_rope(x, w_qkv, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, 20, cfg=28, ss_in=ss),
    }
    gms = (1, 2, 4, 8, 16, 32)
    best = {(k, gm): math.inf for k in cases for gm in gms}
    for _ in range(3):
        for gm in gms:
            ops.gemm_set_group_m(gm)
            for k, fn in cases.items():
                best[(k, gm)] = min(best[(k, gm)], graph_time(fn, 7, 8))
    ops.gemm_set_group_m(8)
    out = {k: {str(gm): round(best[(k, gm)], 1) for gm in gms} for k in cases}
    print(json.dumps({f"M{M}": out}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
