#!/usr/bin/env python3
"""Tile-config sweep of the fused GEMMs at the engine's shapes, interleaved.

kbench.py times configs one after another, so clock ramp and cache state bias
whichever runs first.  Here every round visits every config of a shape once
(round-robin), each visit = median of ``--iters`` replays of a hipGraph of
``--inner`` launches, and a config's time is its best round.  Prints one JSON
object {shape: {cfg: us, "auto": cfg, "best": cfg}}.

    python scripts/gemm_tune.py --rows 9216,4608,16384 --rounds 4
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd import ops  # noqa: E402


def graph_time(fn, iters: int, inner: int) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--rows", default="9216,4608,16384")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--iters", type=int, default=9)
    p.add_argument("--inner", type=int, default=20)
    p.add_argument("--only", default="", help="comma list of shapes (gate_up,down,o,qkv_rope); default all")
    p.add_argument("--cfgs", default="", help="comma list of tile configs to time; default every one that fits")
    a = p.parse_args()
    only = set(filter(None, a.only.split(",")))
    pick = {int(c) for c in a.cfgs.split(",") if c}
    dev = "cuda"
    torch.manual_seed(0)
    H, I, nh, nkv, D = 576, 1536, 9, 3, 64

    def bf(*shape):
        return (torch.randn(*shape, device=dev) * 0.05).to(torch.bfloat16)

    res = {}
    w_gu, w_down, w_o = bf(2 * I, H), bf(H, I), bf(H, H)
    w_qkv = bf((nh + 2 * nkv) * D, H)
    for M in (int(x) for x in a.rows.split(",")):
        x, h = bf(M, H), bf(M, I)
        resid = bf(M, H)
        out_gu = torch.empty(M, I, dtype=torch.bfloat16, device=dev)
        S, Lmax = 8192, 256
        pos = torch.randint(0, 200, (M,), dtype=torch.int32, device=dev)
        slot = torch.randint(0, S, (M,), dtype=torch.int32, device=dev)
        cs = ops.rope_table(1024, D, 1e5, device=dev)
        kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=dev)
        vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=dev)
        q_out = torch.empty(M, nh, D, dtype=torch.bfloat16, device=dev)
        # the engine's flavour: norm GEMMs read the producer's x² partials, residual GEMMs write them
        ss = ops.ss_buffer(M, dev)
        ss[:9] = torch.rand(9, M, device=dev)
        sso = ops.ss_buffer(M, dev)

        def resid_fn(a_, w_):
            def fn(c):
                if H // ops.GEMM_TILES[c][1] > ops.SS_PARTS:
                    raise ValueError("too many N tiles for the partials")
                return ops.gemm(a_, w_, epi="resid", resid=resid, cfg=c, ss_out=sso)
            return fn
        shapes = {
            "gate_up": (2 * I, H, "swiglu",
                        lambda c: ops.gemm(x, w_gu, epi="swiglu", norm_eps=1e-5, out=out_gu, cfg=c, ss_in=ss)),
            "down": (H, I, "resid", resid_fn(h, w_down)),
            "o": (H, H, "resid", resid_fn(x, w_o)),
        }
        for name, (N, K, epi, fn) in shapes.items():
            if only and name not in only:
                continue
            cfgs = [c for c, (bm, bn) in ops.GEMM_TILES.items() if N % bn == 0 and (not pick or c in pick)
                    and not (epi == "swiglu" and c in ops.GEMM_NO_SWIGLU)
                    and not (epi != "swiglu" and c in ops.GEMM_SWIGLU_ONLY)]
            best = {c: math.inf for c in cfgs}
            for _ in range(a.rounds):
                for c in cfgs:
                    try:
                        best[c] = min(best[c], graph_time(lambda: fn(c), a.iters, a.inner))
                    except (RuntimeError, ValueError):
                        best[c] = math.nan
            ok = {c: round(t, 2) for c, t in best.items() if math.isfinite(t)}
            auto = ops.gemm_cfg(M, N, epi=epi, K=K)
            res[f"{name}_M{M}"] = {"us": ok, "auto": auto, "auto_us": ok.get(auto),
                                   "best": min(ok, key=ok.get) if ok else None}
            print(json.dumps({f"{name}_M{M}": res[f"{name}_M{M}"]}), file=sys.stderr, flush=True)
        if not only or "qkv_rope" in only:
            qcfgs = [c for c in (1, 3, 5, 17, 18, 23, 26, 28, 39, 40, 41) if not pick or c in pick]
            best = {c: math.inf for c in qcfgs}
            for _ in range(a.rounds):
                for c in qcfgs:
                    best[c] = min(best[c], graph_time(
                        lambda: ops.gemm_qkv_rope(x, w_qkv, 1e-5, pos, slot, cs, q_out, kc, vt, nh, nkv, 20, cfg=c,
                                                  ss_in=ss),
                        a.iters, a.inner))
            ok = {c: round(t, 2) for c, t in best.items()}
            res[f"qkv_rope_M{M}"] = {"us": ok, "best": min(ok, key=ok.get)}
            print(json.dumps({f"qkv_rope_M{M}": res[f"qkv_rope_M{M}"]}), file=sys.stderr, flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
