"""Scaling probe for the fused GEMM: time vs K (fixed M, N) and vs M (fixed K), plus hipBLASLt."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.kbench import timeit  # noqa: E402
from smsgate_amd import ops  # noqa: E402


def main():
    dev, bf = "cuda", torch.bfloat16
    res = {}
    for K in (64, 128, 256, 576, 1152, 2304):
        X, W = torch.randn(4096, K, device=dev).to(bf), torch.randn(3072, K, device=dev).to(bf) * 0.05
        for c in (0, 1, 3):
            res[f"K{K}_cfg{c}"] = timeit(lambda: ops.gemm(X, W, cfg=c))
        res[f"K{K}_blas"] = timeit(lambda: F.linear(X, W))
    for M in (256, 1024, 2048, 4096, 8192, 16384):
        X, W = torch.randn(M, 576, device=dev).to(bf), torch.randn(3072, 576, device=dev).to(bf) * 0.05
        res[f"M{M}_cfg0"] = timeit(lambda: ops.gemm(X, W, cfg=0))
        res[f"M{M}_blas"] = timeit(lambda: F.linear(X, W))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
