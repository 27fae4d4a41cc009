"""Driver for counter runs: the gate_up GEMM (fused SwiGLU+norm) at batch B for the
tile configs in CFGS, and hipBLASLt on the same shape.  EPI=resid: the N = 576
residual GEMM (o-proj with K=576, down-proj with K=1536) instead."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smsgate_amd import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
B = int(os.environ.get("B", "4096"))
EPI = os.environ.get("EPI", "swiglu")
K = int(os.environ.get("K", "576"))
X = torch.randn(B, K, device=dev).to(bf)
W = (torch.randn(3072 if EPI == "swiglu" else 576, K, device=dev) * 0.05).to(bf)
R = torch.randn(B, 576, device=dev).to(bf)
for cfg in [int(c) for c in os.environ.get("CFGS", os.environ.get("CFG", "0")).split(",")]:
    for _ in range(10):
        if EPI == "swiglu":
            ops.gemm(X, W, epi="swiglu", norm_eps=1e-5, cfg=cfg)
        else:
            ops.gemm(X, W, epi="resid", resid=R, cfg=cfg)
for _ in range(10):
    F.linear(X, W)
torch.cuda.synchronize()
print("ok")
