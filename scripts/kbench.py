"""Per-op microbenchmark of one decode step of the 135M extractor at batch B.

Times every HIP kernel and every projection GEMM at the serving shapes with
CUDA events (median of N replays), plus the whole decode step through the
engine's captured graph, and prints one JSON object.  Usage (GPU box):
    python scripts/kbench.py --batch 2048 --ctx 60
"""
import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd import ops  # noqa: E402
from smsgate_amd.models.extractor import CONFIGS  # noqa: E402


def timeit(fn, iters=15, inner=20, warm=3):
    """GPU time per launch in µs: ``inner`` launches captured in one hipGraph (as
    the engine runs them), median over ``iters`` replays. Includes the ~1 µs
    kernel-boundary cost but not host launch overhead."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(inner):
            fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / inner)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=2048)
    p.add_argument("--ctx", type=int, default=60, help="own keys per sequence")
    p.add_argument("--model", default="smollm-135m")
    a = p.parse_args()
    cfg = CONFIGS[a.model]
    B, H, D, nh, nkv, I, V = a.batch, cfg.hidden, cfg.head_dim, cfg.heads, cfg.kv_heads, cfg.inter, cfg.vocab
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*s):
        return (torch.randn(*s, generator=g) * 0.02).to(bf).to(dev)

    P0, P0pad, Lmax = 75, 96, 192
    res = {}
    x = rnd(B, H)
    w = torch.ones(H, dtype=bf, device=dev)
    res["rmsnorm_residual"] = timeit(lambda: ops.rmsnorm_residual(x, w, 1e-5, x=x))
    gu = rnd(B, 2 * I)
    res["silu_mul"] = timeit(lambda: ops.silu_mul(gu))
    qkv = rnd(B, (nh + 2 * nkv) * D)
    pos = torch.full((B,), a.ctx - 1, dtype=torch.int32, device=dev)
    slot = torch.arange(B, dtype=torch.int32, device=dev)
    kc = rnd(B, nkv, Lmax, D)
    vt = rnd(*ops.vt_shape(B, nkv, D, Lmax))
    pk, pvt = rnd(nkv, P0pad, D), rnd(*ops.vt_shape(1, nkv, D, P0pad)[1:])
    cs = ops.rope_table(P0 + Lmax + 1, D, cfg.rope_theta, dev)
    q = torch.empty(B, nh, D, dtype=bf, device=dev)
    res["rope_qkv_cache"] = timeit(lambda: ops.rope_qkv_cache(qkv, pos, slot, cs, q, kc, vt, nh, nkv, D, P0))
    out = torch.empty(B, nh * D, dtype=bf, device=dev)
    done = torch.zeros(B, dtype=torch.int32, device=dev)
    res["attn_decode"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D),
                                                        done=done, impl="mfma"))
    scr = (torch.empty(B, nh, D, dtype=torch.float32, device=dev), torch.empty(B, nh, dtype=torch.float32, device=dev))
    res["attn_decode_cascade"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out,
                                                                1 / math.sqrt(D), done=done, scratch=scr))
    res["attn_decode_st"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D),
                                                           done=done, impl="mfma"))
    res["attn_decode_v1"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D),
                                                           done=done, impl="mfma_v1"))
    res["attn_decode_valu"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out,
                                                             1 / math.sqrt(D), done=done, impl="valu"))
    for impl in ("grouped", "grouped_h", "grouped6", "grouped_pf", "split2", "split4", "split8"):
        res[f"attn_decode_{impl}"] = timeit(lambda: ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out,
                                                                    1 / math.sqrt(D), done=done, impl=impl))
    kv_bytes = B * nkv * a.ctx * D * 2 * 2
    res["attn_decode_own_kv_GBps"] = round(kv_bytes / (res["attn_decode"] * 1e-6) / 1e9, 1)
    for name, (n, k) in {"qkv": (cfg.qkv_out, H), "o": (H, nh * D), "gate_up": (2 * I, H), "down": (H, I),
                         "lm_head": (V, H)}.items():
        W = rnd(n, k)
        X = rnd(B, k)
        t = timeit(lambda: F.linear(X, W))
        res[f"gemm_{name}"] = t
        res[f"gemm_{name}_TFLOPs"] = round(2 * B * n * k / (t * 1e-6) / 1e12, 1)
    # fused MFMA GEMMs (csrc/gemm_kernels.hip) at the same shapes, every tile config
    fused = {"qkv": (cfg.qkv_out, H, "store", True), "o": (H, nh * D, "resid", False),
             "gate_up": (2 * I, H, "swiglu", True), "down": (H, I, "resid", False),
             "lm_head": (8192, H, "store", True)}
    for name, (n, k, epi, norm) in fused.items():
        W = rnd(n, k)
        X = rnd(B, k)
        R = rnd(B, n) if epi == "resid" else None
        kw = dict(epi=epi, norm_eps=1e-5 if norm else None, resid=R)
        best = None
        for c, (bm, bn) in ops.GEMM_TILES.items():
            if n % bn or (c in ops.GEMM_SWIGLU_ONLY and epi != "swiglu"):
                continue
            t = timeit(lambda: ops.gemm(X, W, cfg=c, **kw))
            res[f"fgemm_{name}_cfg{c}"] = t
            best = t if best is None else min(best, t)
        res[f"fgemm_{name}_auto"] = timeit(lambda: ops.gemm(X, W, **kw))
        res[f"fgemm_{name}_auto_cfg"] = ops.gemm_cfg(B, n)
        res[f"fgemm_{name}_TFLOPs"] = round(2 * B * n * k / (best * 1e-6) / 1e12, 1)
    Xl, Wl = rnd(B, H), rnd(8192, H)
    res["gemm_lm_head_8192"] = timeit(lambda: F.linear(Xl, Wl))
    # QKV projection + RoPE + KV scatter: fused epilogue vs GEMM + separate kernel
    Xq, Wq = rnd(B, H), rnd(cfg.qkv_out, H)
    qo = torch.empty(B, nh, D, dtype=bf, device=dev)
    for c in (1, 3, 5, 17, 18):
        res[f"qkv_rope_fused_cfg{c}"] = timeit(lambda: ops.gemm_qkv_rope(Xq, Wq, 1e-5, pos, slot, cs, qo, kc, vt, nh, nkv,
                                                                          P0, cfg=c))
    res["qkv_rope_fused_auto"] = timeit(lambda: ops.gemm_qkv_rope(Xq, Wq, 1e-5, pos, slot, cs, qo, kc, vt, nh, nkv, P0))
    res["qkv_rope_split"] = timeit(lambda: ops.rope_qkv_cache(ops.gemm(Xq, Wq, norm_eps=1e-5), pos, slot, cs, qo, kc, vt,
                                                               nh, nkv, D, P0))
    fused_layer = (res["rope_qkv_cache"] + res["attn_decode_cascade"] + res["fgemm_qkv_auto"] + res["fgemm_o_auto"]
                   + res["fgemm_gate_up_auto"] + res["fgemm_down_auto"])
    res["fused_sum_per_layer_us"] = round(fused_layer, 1)
    res["fused_est_step_us"] = round(fused_layer * cfg.layers + res["fgemm_lm_head_auto"], 1)
    per_layer = (2 * res["rmsnorm_residual"] + res["rope_qkv_cache"] + res["attn_decode"] + res["silu_mul"]
                 + res["gemm_qkv"] + res["gemm_o"] + res["gemm_gate_up"] + res["gemm_down"])
    res["sum_per_layer_us"] = round(per_layer, 1)
    res["est_step_us"] = round(per_layer * cfg.layers + res["gemm_lm_head"], 1)
    res["batch"], res["ctx"] = B, a.ctx
    print(json.dumps(res))


if __name__ == "__main__":
    main()
