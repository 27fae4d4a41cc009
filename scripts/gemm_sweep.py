"""Fused-GEMM tile-config sweep on the extractor's decode shapes (and hipBLASLt).

python scripts/gemm_sweep.py [--batch 8192,4096] [--cfgs 0,1,9] → one JSON line per batch:
{shape: {cfg: us, "blas": us, "best": cfg, "TFLOPs": x}}."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.kbench import timeit  # noqa: E402
from smsgate_amd import ops  # noqa: E402

SHAPES = {"qkv": (960, 576, "store", True), "o": (576, 576, "resid", False),
          "gate_up": (3072, 576, "swiglu", True), "down": (576, 1536, "resid", False),
          "lm_head": (8192, 576, "store", True)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="8192")
    ap.add_argument("--cfgs", default="")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--group-m", default="8", help="rasterisation groups to sweep")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else sorted(ops.GEMM_TILES)
    dev, bf = "cuda", torch.bfloat16
    for B in [int(b) for b in a.batch.split(",")]:
        out = {"batch": B}
        for name in a.shapes.split(","):
            n, k, epi, norm = SHAPES[name]
            X = torch.randn(B, k, device=dev).to(bf)
            W = (torch.randn(n, k, device=dev) * k ** -0.5).to(bf)
            R = torch.randn(B, n, device=dev).to(bf) if epi == "resid" else None
            kw = dict(epi=epi, norm_eps=1e-5 if norm else None, resid=R)
            r = {}
            for gm in [int(g) for g in a.group_m.split(",")]:
                ops.gemm_set_group_m(gm)
                for c in cfgs:
                    bm, bn = ops.GEMM_TILES[c]
                    if n % bn or (c in ops.GEMM_SWIGLU_ONLY and epi != "swiglu"):
                        continue
                    r[f"{c}/g{gm}"] = timeit(lambda: ops.gemm(X, W, cfg=c, **kw))
            r["blas"] = timeit(lambda: F.linear(X, W))
            best = min((v, c) for c, v in r.items() if c != "blas")
            r["best"] = best[1]
            r["TFLOPs"] = round(2 * B * n * k / (best[0] * 1e-6) / 1e12, 1)
            out[name] = r
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
