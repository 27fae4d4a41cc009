#!/usr/bin/env python3
"""Cost of the fused RMSNorm prologue in the GEMMs: the same GEMM with and without
NORM (row sum of squares accumulated with v_dot2 beside the MFMAs) at the engine's
verify-step shapes.  Prints one JSON object {shape: {"norm": us, "plain": us}}."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd import ops  # noqa: E402
from scripts.gemm_tune import graph_time  # noqa: E402


def main() -> None:
    ops.load_library()
    dev = "cuda"
    out = {}
    for M in (4608, 9216):
        for name, N, K, epi, cfgs in (("gate_up", 3072, 576, "swiglu", (0, 10)), ("qkv", 960, 576, "store", (1, 3)),
                                      ("lm", 8192, 576, "store", (0,))):
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
            for cfg in cfgs:
                row = {}
                ssb = ops.ss_buffer(M, dev)
                ssb[:9] = torch.rand(9, M, device=dev) * 50
                for tag, eps, si in (("norm", 1e-5, None), ("plain", None, None), ("ssin", 1e-5, ssb if epi == "swiglu" else None)):
                    fn = lambda: ops.gemm(a, w, epi=epi, norm_eps=eps, cfg=cfg, ss_in=si)  # noqa: E731
                    row[tag] = round(min(graph_time(fn, 20, 20) for _ in range(3)), 2)
                row["tflops_plain"] = round(2 * M * N * K / row["plain"] / 1e6, 1)
                out[f"{name} M={M} cfg={cfg}"] = row
                print(f"{name} M={M} cfg={cfg} {row}", flush=True)
    # epilogue costs at the verify step's 9216 rows: QKV + RoPE + KV scatter vs a plain
    # store; residual GEMMs with / without the x² partials for the next norm
    M, H, I, nh, nkv, S, Lmax = 9216, 576, 1536, 9, 3, 8193, 192
    x = torch.randn(M, H, device=dev).to(torch.bfloat16)
    wq = (torch.randn((nh + 2 * nkv) * 64, H, device=dev) * 0.05).to(torch.bfloat16)
    pos = torch.randint(0, 60, (M,), device=dev, dtype=torch.int32)
    slot = torch.randint(0, S, (M,), device=dev, dtype=torch.int32)
    cs = ops.rope_table(20 + Lmax + 1, 64, 100000.0, dev)
    q = torch.empty(M, nh, 64, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(S, nkv, Lmax, 64, dtype=torch.bfloat16, device=dev)
    vt = torch.zeros(*ops.vt_shape(S, nkv, 64, Lmax), dtype=torch.bfloat16, device=dev)
    ss = ops.ss_buffer(M, dev)
    ss[:9] = torch.rand(9, M, device=dev) * 500
    for cfg in (1, 3):
        row = {}
        row["store_norm"] = round(min(graph_time(lambda: ops.gemm(x, wq, norm_eps=1e-5, cfg=cfg), 20, 20)
                                      for _ in range(3)), 2)
        row["rope_norm"] = round(min(graph_time(lambda: ops.gemm_qkv_rope(
            x, wq, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, 20, cfg=cfg), 20, 20) for _ in range(3)), 2)
        row["rope_ssin"] = round(min(graph_time(lambda: ops.gemm_qkv_rope(
            x, wq, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, 20, cfg=cfg, ss_in=ss), 20, 20) for _ in range(3)), 2)
        out[f"qkv_rope M={M} cfg={cfg}"] = row
        print(f"qkv_rope M={M} cfg={cfg} {row}", flush=True)
    for name, K in (("o_proj", H), ("down", I)):
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(H, K, device=dev) * 0.05).to(torch.bfloat16)
        r = torch.randn(M, H, device=dev).to(torch.bfloat16)
        for cfg in (1, 3):
            row = {}
            sso = ops.ss_buffer(M, dev)
            row["resid"] = round(min(graph_time(lambda: ops.gemm(a, w, epi="resid", resid=r, cfg=cfg), 20, 20)
                                     for _ in range(3)), 2)
            row["resid_ssout"] = round(min(graph_time(lambda: ops.gemm(a, w, epi="resid", resid=r, cfg=cfg,
                                                                       ss_out=sso), 20, 20) for _ in range(3)), 2)
            row["tflops"] = round(2 * M * H * K / row["resid"] / 1e6, 1)
            out[f"{name} M={M} cfg={cfg}"] = row
            print(f"{name} M={M} cfg={cfg} {row}", flush=True)
    # lm_head + FSM-masked arg-max (EPI 4) against the same GEMM storing logits
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import build_fsm

    tk = load_tokenizer()
    V = (tk.vocab_size + 127) // 128 * 128
    fsm = build_fsm(tk, V).to_device(dev)
    wl = (torch.randn(V, H, device=dev) * 0.05).to(torch.bfloat16)
    st = torch.randint(0, fsm.num_states, (M,), device=dev, dtype=torch.int32)
    best = torch.zeros(M, dtype=torch.int64, device=dev)
    row = {"store_norm_cfg0": round(min(graph_time(lambda: ops.gemm(x, wl, norm_eps=1e-5, cfg=0), 20, 10)
                                        for _ in range(3)), 2)}
    for cfg in (0, 3):
        row[f"argmax_ssin_cfg{cfg}"] = round(min(graph_time(lambda: ops.gemm_argmax(
            x, wl, st, fsm, best, norm_eps=1e-5, cfg=cfg, ss_in=ss), 20, 10) for _ in range(3)), 2)
    out[f"lm_argmax M={M} V={V}"] = row
    print(f"lm_argmax M={M} V={V} {row}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
