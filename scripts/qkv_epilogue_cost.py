#!/usr/bin/env python3
"""What the QKV+RoPE GEMM's epilogue costs at the qa engine's batch sizes: the same
[M, 576] x [960, 576]^T product with a plain bf16 store (EPI 0) vs the fused
RoPE + q write + K / V^T cache scatter (EPI 3), each tile config that fits, graph-timed
(scripts/gemm_tune.py graph_time), interleaved rounds."""
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
    H, nh, nkv, D, S, Lmax = 576, 9, 3, 64, 8192, 160
    N = (nh + 2 * nkv) * D
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*shape):
        return (torch.randn(*shape, generator=g) * 0.05).to(bf16).to(dev)

    w = bf(N, H)
    cs = ops.rope_table(1024, D, 1e5, device=dev)
    kc = bf(S, nkv, Lmax, D)
    vt = bf(*ops.vt_shape(S, nkv, D, Lmax))
    out = {}
    for M in (110592, 221184):
        x = bf(M, H)
        ss = ops.ss_buffer(M, dev)
        ss[:6] = torch.rand(6, M, device=dev)
        pos = torch.randint(0, 120, (M,), generator=g, dtype=torch.int32).to(dev)
        slot = torch.randint(0, S, (M,), generator=g, dtype=torch.int32).to(dev)
        # the engine's layout: packed sequences of ~50 rows, positions 0.. within each, one
        # KV slot per sequence (whole 8-position V^T blocks)
        r = torch.arange(M, dtype=torch.int32)
        ppos, pslot = (r % 50).to(dev), ((r // 50) % S).to(dev)
        q = torch.empty(M, nh, D, dtype=bf16, device=dev)
        c = torch.empty(M, N, dtype=bf16, device=dev)
        cases = {
            # NORM 1 (x² in the K loop) on both sides: plain store vs the fused epilogue
            "store_n1_cfg28": lambda: ops.gemm(x, w, norm_eps=1e-5, out=c, cfg=28),
            "rope_n1_cfg28_packed": lambda: ops.gemm_qkv_rope(x, w, 1e-5, ppos, pslot, cs, q, kc, vt, nh, nkv, 20,
                                                              cfg=28),
            "rope_n1_cfg28_random": lambda: ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, 20,
                                                              cfg=28),
            # the engine's flavour (producer partials)
            "rope_n2_cfg28_packed": lambda: ops.gemm_qkv_rope(x, w, 1e-5, ppos, pslot, cs, q, kc, vt, nh, nkv, 20,
                                                              cfg=28, ss_in=ss),
        }
        best = {}
        for k, fn in list(cases.items()):
            try:
                fn()
                torch.cuda.synchronize()
                best[k] = math.inf
            except Exception as exc:  # noqa: BLE001 -- a config this epilogue has no instance of
                print(json.dumps({"skip": k, "why": str(exc)[:120]}), flush=True)
                cases.pop(k)
        for _ in range(3):
            for k, fn in cases.items():
                best[k] = min(best[k], graph_time(fn, 7, 8))
        fl = 2.0 * M * N * H
        out[f"M{M}"] = {k: {"us": round(v, 1), "tflops": round(fl / v / 1e6, 1)} for k, v in best.items()}
        print(json.dumps({f"M{M}": out[f"M{M}"]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
