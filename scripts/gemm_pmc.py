"""Driver for counter runs: the gate_up GEMM (fused SwiGLU+norm) at batch B for the
tile configs in CFGS, and hipBLASLt on the same shape."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smsgate_amd import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
B = int(os.environ.get("B", "4096"))
X = torch.randn(B, 576, device=dev).to(bf)
W = (torch.randn(3072, 576, device=dev) * 0.05).to(bf)
for cfg in [int(c) for c in os.environ.get("CFGS", os.environ.get("CFG", "0")).split(",")]:
    for _ in range(10):
        ops.gemm(X, W, epi="swiglu", norm_eps=1e-5, cfg=cfg)
for _ in range(10):
    F.linear(X, W)
torch.cuda.synchronize()
print("ok")
