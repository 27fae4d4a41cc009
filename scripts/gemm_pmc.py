"""Driver for counter runs: the gate_up GEMM at B=4096 (fused SwiGLU+norm) and hipBLASLt."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smsgate_amd import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
X = torch.randn(4096, 576, device=dev).to(bf)
W = (torch.randn(3072, 576, device=dev) * 0.05).to(bf)
for _ in range(10):
    ops.gemm(X, W, epi="swiglu", norm_eps=1e-5, cfg=int(os.environ.get("CFG", "0")))
for _ in range(10):
    F.linear(X, W)
torch.cuda.synchronize()
print("ok")
