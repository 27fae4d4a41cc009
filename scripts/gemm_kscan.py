#!/usr/bin/env python3
"""Fixed vs per-K-tile cost of the SwiGLU GEMMs: time at several K (same M, N); a
straight-line fit time = a + b·(K/64) separates prologue/epilogue (a) from the K loop (b)."""
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
    dev, M, N = "cuda", 9216, 3072
    out = {}
    for cfg in (0, 19, 20):
        pts = []
        for K in (576, 1152, 2304, 4608):
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
            t = min(graph_time(lambda: ops.gemm(a, w, epi="swiglu", cfg=cfg), 20, 10) for _ in range(3))
            pts.append((K // 64, t))
        n = len(pts)
        sx = sum(p[0] for p in pts); sy = sum(p[1] for p in pts)
        sxx = sum(p[0] ** 2 for p in pts); sxy = sum(p[0] * p[1] for p in pts)
        b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
        a = (sy - b * sx) / n
        tiles = -(-M // ops.GEMM_TILES[cfg][0]) * (N // ops.GEMM_TILES[cfg][1])
        out[f"cfg{cfg}"] = {"us": {k * 64: round(t, 2) for k, t in pts}, "fixed_us": round(a, 2),
                            "per_ktile_us": round(b, 3), "tiles": tiles,
                            "loop_tflops": round(2 * M * N * 64 / b / 1e6, 1)}
        print(cfg, out[f"cfg{cfg}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
