"""Time decomposition of the fused GEMM K loop (sg_gemm_probe): full kernel vs
loads-only vs MFMA-only, for the SwiGLU+norm shape at several batches."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.kbench import timeit  # noqa: E402
from smsgate_amd import ops  # noqa: E402
from smsgate_amd.ops import _p, _stream, load_library  # noqa: E402

lib = load_library()
out = {}
for B in (4096, 8192):
    for K in (576, 1536):
        N = 3072
        X = torch.randn(B, K, device="cuda").to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") * 0.03).to(torch.bfloat16)
        C = torch.empty(B, N // 2, device="cuda", dtype=torch.bfloat16)
        r = {}
        for mode, name in ((0, "full"), (1, "loads_only"), (2, "mfma_only"), (3, "mfma_no_prologue"),
                           (4, "mfma_no_prologue_no_epilogue")):
            r[name] = timeit(lambda: lib.sg_gemm_probe(_p(X), _p(W), _p(C), B, N, K, mode, _stream()))
        r["mfma_bound_us"] = round(2 * B * N * K / 2.5e15 * 1e6, 2)
        out[f"B{B}_K{K}"] = r
print(json.dumps(out))
