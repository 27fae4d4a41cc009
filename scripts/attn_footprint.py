"""Does decode attention at large batch pay for KV *footprint* (TLB / cache)?  Same work
(B rows, ctx keys each), slots drawn from a pool of P distinct KV slots."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.kbench import timeit  # noqa: E402
from smsgate_amd import ops  # noqa: E402


def main():
    dev, bf = "cuda", torch.bfloat16
    nh, nkv, D, P0, P0pad, ctx = 9, 3, 64, 75, 96, 75
    res = {}
    for B, pool, Lmax in ((4096, 4096, 192), (8192, 8192, 192), (16384, 16384, 192)):
        q = (torch.randn(B, nh, D, device=dev) * 0.1).to(bf)
        kc = (torch.randn(pool, nkv, Lmax, D, device=dev) * 0.1).to(bf)
        vt = (torch.randn(*ops.vt_shape(pool, nkv, D, Lmax), device=dev) * 0.1).to(bf)
        pk = (torch.randn(nkv, P0pad, D, device=dev) * 0.1).to(bf)
        pvt = (torch.randn(*ops.vt_shape(1, nkv, D, P0pad)[1:], device=dev) * 0.1).to(bf)
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
        slot = (torch.arange(B, device=dev) % pool).to(torch.int32)
        out = torch.empty(B, nh * D, dtype=bf, device=dev)
        done = torch.zeros(B, dtype=torch.int32, device=dev)
        scr = (torch.empty(B, nh, D, dtype=torch.float32, device=dev), torch.empty(B, nh, dtype=torch.float32, device=dev))
        for impl in ("cascade", "grouped"):
            res[f"{impl}_B{B}_pool{pool}_L{Lmax}"] = timeit(lambda: ops.attn_decode(
                q, pos, slot, kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D), done=done, scratch=scr, impl=impl))
        del kc, vt
    print(json.dumps(res))


if __name__ == "__main__":
    main()
