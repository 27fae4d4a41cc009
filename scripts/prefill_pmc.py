"""Driver for counter runs of the prefill attention at the engine's shape (one
prefill half: ~8 k tokens of 150-200 sequences, 21-token shared prefix); IMPL picks
the kernel (per_head / multi / gqa)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smsgate_amd import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
NSEQ = int(os.environ.get("NSEQ", "190"))
IMPL = os.environ.get("IMPL", "per_head")
ITERS = int(os.environ.get("ITERS", "20"))
nh, nkv, D, P0, Lmax = 9, 3, 64, 21, 288
P0pad = 32
g = torch.Generator(device="cpu").manual_seed(0)
lens = torch.randint(30, 56, (NSEQ,), generator=g).tolist()
T = sum(lens)


def rnd(*s):
    return (torch.randn(*s, generator=g) * 0.5).to(bf).to(dev)


q = rnd(T, nh, D)
kc = rnd(NSEQ, nkv, Lmax, D)
vt = rnd(*ops.vt_shape(NSEQ, nkv, D, Lmax))
pk, pvt = rnd(nkv, P0pad, D), rnd(*ops.vt_shape(1, nkv, D, P0pad)[1:])
cu = torch.tensor([0] + torch.cumsum(torch.tensor(lens), 0).tolist(), dtype=torch.int32, device=dev)
qs = torch.zeros(NSEQ, dtype=torch.int32, device=dev)
sl = torch.arange(NSEQ, dtype=torch.int32, device=dev)
out = torch.empty(T, nh * D, dtype=bf, device=dev)
ops.set_prefill_impl(IMPL)
for _ in range(ITERS):
    ops.attn_prefill(q, cu, qs, sl, max(lens), kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D))
torch.cuda.synchronize()
print(T, NSEQ, IMPL)
