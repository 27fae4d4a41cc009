#!/usr/bin/env python3
"""The staggered 256x256 SwiGLU GEMM (cfg 19) against the 128x128 kernel (cfg 0), the
8-wave 256x256 two-barrier kernel (cfg 10) and the fp32 reference: max errors, then
interleaved timings at the engine's row counts (NORM 1 and producer row partials)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd import ops  # noqa: E402
from scripts.gemm_tune import graph_time  # noqa: E402


def main() -> None:
    ops.load_library()
    dev = "cuda"
    out = {"check": {}, "time": {}}
    torch.manual_seed(0)
    for M, K in ((5, 576), (640, 576), (2000, 1536), (9216, 576)):
        I = 1536
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        nw = (torch.randn(K, device=dev) * 0.1 + 1).to(torch.bfloat16)
        gu = (torch.randn(2 * I, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        w = ops.interleave_gate_up(ops.fold_norm(gu, nw))
        ref = ops.ref_gemm(a, gu, epi="swiglu", norm_eps=1e-5, norm_w=nw)
        o19 = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=19).float()
        o20 = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=20).float()
        ss = ops.ss_buffer(M, dev)
        ss[0, :M] = a.float().pow(2).sum(1)
        o20s = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=20, ss_in=ss).float()
        o0 = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=0).float()
        rec = {"max_err_ref": float((o19 - ref).abs().max()), "max_err_cfg0_ref": float((o0 - ref).abs().max()),
               "max_diff_cfg0": float((o19 - o0).abs().max()), "max_diff_cfg20": float((o20 - o0).abs().max()),
               "max_err_cfg20_ssin_ref": float((o20s - ref).abs().max())}
        out["check"][f"M={M} K={K}"] = rec
        print("check", M, K, rec, flush=True)
    for M in (4608, 9216, 16384):
        K, N = 576, 3072
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        ss = ops.ss_buffer(M, dev)
        ss[:9] = torch.rand(9, M, device=dev) * 50
        res = {}
        for rnd in range(3):
            for cfg in (0, 10, 19, 20):
                for tag, si in (("ssin", ss), ("norm", None)):
                    t = graph_time(lambda: ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=cfg, ss_in=si), 20, 20)
                    k = f"cfg{cfg}_{tag}"
                    res[k] = round(min(res.get(k, 1e9), t), 2)
        res["tflops_cfg20_ssin"] = round(2 * M * N * K / res["cfg20_ssin"] / 1e6, 1)
        out["time"][f"M={M}"] = res
        print("time", M, res, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
