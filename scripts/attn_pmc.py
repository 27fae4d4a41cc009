"""Driver for counter runs of the decode attention (grouped kernel, the default):
B rows with CTX own keys each plus the 75-token shared prefix, at the 135M
extractor's head shape.  Prints the bytes the kernel must read (own K+V, prefix
K+V once) so the FETCH_SIZE counter can be compared against it."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smsgate_amd import ops  # noqa: E402

dev, bf = "cuda", torch.bfloat16
B = int(os.environ.get("B", "4096"))
CTX = int(os.environ.get("CTX", "72"))
IMPL = os.environ.get("IMPL", "grouped")
ITERS = int(os.environ.get("ITERS", "10"))
nh, nkv, D, P0, P0pad, Lmax = 9, 3, 64, 75, 96, 192
g = torch.Generator(device="cpu").manual_seed(0)


def rnd(*s):
    return (torch.randn(*s, generator=g) * 0.02).to(bf).to(dev)


q = rnd(B, nh, D)
pos = torch.full((B,), CTX - 1, dtype=torch.int32, device=dev)
slot = torch.arange(B, dtype=torch.int32, device=dev)
kc = rnd(B, nkv, Lmax, D)
vt = rnd(*ops.vt_shape(B, nkv, D, Lmax))
pk, pvt = rnd(nkv, P0pad, D), rnd(*ops.vt_shape(1, nkv, D, P0pad)[1:])
out = torch.empty(B, nh * D, dtype=bf, device=dev)
done = torch.zeros(B, dtype=torch.int32, device=dev)
for _ in range(ITERS):
    ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D), done=done, impl=IMPL)
torch.cuda.synchronize()
own = B * nkv * CTX * D * 2 * 2
print(json.dumps({"B": B, "ctx": CTX, "impl": IMPL, "own_kv_bytes": own, "q_out_bytes": 2 * B * nh * D * 2,
                  "prefix_bytes": nkv * P0 * D * 2 * 2}))
