"""Fused training forward of the extractor LM (the bench trains it in-run, untimed).

:func:`~smsgate_amd.models.extractor.reference_forward` is the plain-PyTorch forward:
every RMSNorm, RoPE and SwiGLU is a chain of small elementwise kernels forward and
backward (~45 launches per layer), which at the bench recipe (128 sequences x ~60
tokens, 7.7 k rows) spent over half of a training step's GPU time re-reading the same
activations (scripts/train_step_profile.py).  :func:`fused_forward` is the same
network with those groups as single HIP kernels (ops/csrc/train_kernels.hip), each an
autograd Function with a hand-written backward:

* ``RMSNorm``: fp32 residual stream in, bf16 normalised rows out (the GEMM's input, so
  autocast's cast is folded in), rstd saved; backward dx in fp32 and dw from per-block
  partial sums;
* ``RopeSplit``: the QKV GEMM's bf16 output -> q / k / v in SDPA's [B, heads, T, D]
  layout with rotate-half RoPE on q and k (fp32 math, the caller's cos / sin tables);
  backward is the adjoint rotation straight into dqkv;
* ``SwiGLU``: silu(gate) * up from the fused gate/up GEMM output, and its backward;
* ``Attention`` (opt-in, ``SMSGATE_TRAIN_SDPA=own``): causal grouped-query attention over
  the batch (<= 192 rows) straight into the o-proj's [B, T, heads * 64] input and its
  backward -- correct (fp32-reference tests) but one thread per row is latency-bound:
  56 ms of a step against SDPA's ~6 (``r05_train_step_sdpa_ab.jsonl``), so SDPA (flash)
  stays the default.

GEMMs stay hipBLASLt (autocast bf16), so the math is
reference_forward's up to bf16 rounding order (tests/test_train_ops_gpu.py compares
losses and gradients).  CPU / no-library: reference_forward.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from .extractor import ExtractorWeights, _rope_tables

__all__ = ["fused_forward", "rms_norm", "rope_split", "swiglu", "attention", "available", "ATTN_MAX_T"]


def available(device) -> bool:
    return str(device).startswith("cuda") and torch.cuda.is_available()


def _lib():
    return ops.load_library()


def _st() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ok(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name} failed (rc={rc})")


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        if x2.dtype != torch.float32 or not x2.is_contiguous() or w.dtype != torch.float32:
            raise ValueError("rms_norm: contiguous fp32 rows and fp32 weight")
        R = x2.shape[0]
        y = torch.empty(R, H, dtype=torch.bfloat16, device=x.device)
        rstd = torch.empty(R, dtype=torch.float32, device=x.device)
        _ok(_lib().sg_rms_fwd(x2.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), R, H, float(eps), _st()),
            "rms_fwd")
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], H)

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x2, w, rstd = ctx.saved_tensors
        R, H = x2.shape
        dy = dy.reshape(R, H)
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        dy = dy.contiguous()
        rpb = 64
        nb = (R + rpb - 1) // rpb
        dx = torch.empty(R, H, dtype=torch.float32, device=x2.device)
        part = torch.empty(nb, H, dtype=torch.float32, device=x2.device)
        _ok(_lib().sg_rms_bwd(dy.data_ptr(), x2.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                              part.data_ptr(), R, H, rpb, _st()), "rms_bwd")
        return dx.view(ctx.shape), part.sum(0), None


class _RopeSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, nh: int, nkv: int, rep: int):
        B, T, N = qkv.shape
        D = N // (nh + 2 * nkv)
        if qkv.dtype != torch.bfloat16 or D != 64 or N != (nh + 2 * nkv) * D:
            raise ValueError("rope_split: bf16 [B, T, (nh + 2 nkv) * 64]")
        qkv = qkv.contiguous()
        q = torch.empty(B, nh, T, D, dtype=qkv.dtype, device=qkv.device)
        k = torch.empty(B, nkv * rep, T, D, dtype=qkv.dtype, device=qkv.device)
        v = torch.empty(B, nkv * rep, T, D, dtype=qkv.dtype, device=qkv.device)
        _ok(_lib().sg_rope_split(1, qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cos.data_ptr(),
                                 sin.data_ptr(), B, T, nh, nkv, D, rep, _st()), "rope_split")
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, T, nh, nkv, D, rep)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        B, T, nh, nkv, D, rep = ctx.dims
        dev = cos.device

        def _g(t, h):
            if t is None:
                return torch.zeros(B, h, T, D, dtype=torch.bfloat16, device=dev)
            return t.to(torch.bfloat16).contiguous()

        dq, dk, dv = _g(dq, nh), _g(dk, nkv * rep), _g(dv, nkv * rep)
        dqkv = torch.empty(B, T, (nh + 2 * nkv) * D, dtype=torch.bfloat16, device=dev)
        _ok(_lib().sg_rope_split(-1, dqkv.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), cos.data_ptr(),
                                 sin.data_ptr(), B, T, nh, nkv, D, rep, _st()), "rope_split_bwd")
        return dqkv, None, None, None, None, None


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu: torch.Tensor) -> torch.Tensor:
        I2 = gu.shape[-1]
        if gu.dtype != torch.bfloat16 or I2 % 16:
            raise ValueError("swiglu: bf16 [..., 2 I] with I % 8 == 0")
        g2 = gu.reshape(-1, I2).contiguous()
        R, I = g2.shape[0], I2 // 2
        a = torch.empty(R, I, dtype=gu.dtype, device=gu.device)
        _ok(_lib().sg_swiglu_fwd(g2.data_ptr(), a.data_ptr(), R, I, _st()), "swiglu_fwd")
        ctx.save_for_backward(g2)
        ctx.shape = gu.shape
        return a.view(*gu.shape[:-1], I)

    @staticmethod
    def backward(ctx, da: torch.Tensor):
        (g2,) = ctx.saved_tensors
        R, I2 = g2.shape
        da = da.reshape(R, I2 // 2).to(torch.bfloat16).contiguous()
        dgu = torch.empty_like(g2)
        _ok(_lib().sg_swiglu_bwd(da.data_ptr(), g2.data_ptr(), dgu.data_ptr(), R, I2 // 2, _st()), "swiglu_bwd")
        return dgu.view(ctx.shape)


ATTN_MAX_T = 192  # csrc/train_kernels.hip AT_MAXT


class _Attention(torch.autograd.Function):
    """Causal grouped-query attention of one training batch (attn_train_* kernels):
    q [B, nh, T, 64], k / v [B, nkv, T, 64] -> out [B, T, nh * 64] (the o-proj input)."""

    @staticmethod
    def forward(ctx, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float) -> torch.Tensor:
        B, nh, T, D = q.shape
        nkv = k.shape[1]
        if D != 64 or T > ATTN_MAX_T or nh % nkv or q.dtype != torch.bfloat16:
            raise ValueError("attention: bf16, head_dim 64, T <= 192, nh % nkv == 0")
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty(B, T, nh * D, dtype=q.dtype, device=q.device)
        lse = torch.empty(B, nh, T, dtype=torch.float32, device=q.device)
        _ok(_lib().sg_attn_train_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(), B, T,
                                     nh, nkv, float(scale), _st()), "attn_train_fwd")
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout: torch.Tensor):
        q, k, v, out, lse = ctx.saved_tensors
        B, nh, T, D = q.shape
        nkv = k.shape[1]
        dout = dout.to(torch.bfloat16).contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dsum = torch.empty(B, nh, T, dtype=torch.float32, device=q.device)
        _ok(_lib().sg_attn_train_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(),
                                     dout.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dsum.data_ptr(), B,
                                     T, nh, nkv, float(ctx.scale), _st()), "attn_train_bwd")
        return dq, dk, dv, None


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float) -> torch.Tensor:
    return _Attention.apply(q, k, v, scale)


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    return _RMSNorm.apply(x, w, eps)


def rope_split(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, nh: int, nkv: int, rep: int = 1):
    """q [B, nh, T, D], k / v [B, nkv * rep, T, D] (``rep`` copies of each kv head)."""
    return _RopeSplit.apply(qkv, cos, sin, nh, nkv, rep)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    return _SwiGLU.apply(gu)


def fused_forward(w: ExtractorWeights, ids: torch.Tensor, add_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Final-normed hidden states [B, T, H] (bf16) of ``reference_forward(w, ids,
    return_hidden=True, add_ids=add_ids)``; call under ``torch.autocast(bf16)`` with fp32
    master weights (models/train.py)."""
    cfg = w.cfg
    B, T = ids.shape
    nh, nkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
    x = F.embedding(ids, w.embed)
    if add_ids is not None:
        x = x + F.embedding(add_ids.clamp(min=0), w.embed) * (add_ids >= 0).unsqueeze(-1).to(x.dtype)
    x = x.float().contiguous()
    cos, sin = _rope_tables(T, D, cfg.rope_theta, ids.device)
    cos, sin = cos.reshape(T, D // 2).contiguous(), sin.reshape(T, D // 2).contiguous()
    scale = 1.0 / math.sqrt(D)
    # attention: SDPA (flash) by default; SMSGATE_TRAIN_SDPA=own runs the attn_train_*
    # kernels (<= 192 rows; correct, but 56 vs ~6 ms per step: one thread per row is
    # latency-bound, r05_train_step_sdpa_ab.jsonl); the efficient backend has no GQA
    # support, so it gets k / v expanded to nh heads by rope_split (its adjoint sums them)
    sdpa = os.environ.get("SMSGATE_TRAIN_SDPA", "")
    rep = nh // nkv if sdpa == "efficient" else 1
    own = sdpa == "own" and T <= ATTN_MAX_T
    with _sdpa_backend():
        for i in range(cfg.layers):
            x = _layer(w, i, x, cos, sin, scale, B, T, nh, nkv, D, rep, own)
    return rms_norm(x, w.ln_f, cfg.eps)


def _sdpa_backend():
    """SMSGATE_TRAIN_SDPA = flash | efficient | math pins SDPA's backend (A/B of the
    training step, scripts/train_step_profile.py); default: PyTorch's choice."""
    name = os.environ.get("SMSGATE_TRAIN_SDPA", "")
    if name in ("", "own"):
        return contextlib.nullcontext()
    from torch.nn.attention import SDPBackend, sdpa_kernel

    return sdpa_kernel({"flash": SDPBackend.FLASH_ATTENTION, "efficient": SDPBackend.EFFICIENT_ATTENTION,
                        "math": SDPBackend.MATH}[name])


def _layer(w, i, x, cos, sin, scale, B, T, nh, nkv, D, rep=1, own=False):
    """One decoder layer of the residual stream ``x`` (fp32)."""
    eps = w.cfg.eps
    h = rms_norm(x, w.ln1[i], eps)
    q, k, v = rope_split(h @ w.qkv[i].t(), cos, sin, nh, nkv, rep)
    if own:
        a = attention(q, k, v, scale)
    else:
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale,
                                           enable_gqa=nh != nkv * rep).transpose(1, 2).reshape(B, T, nh * D)
    x = x + a @ w.o[i].t()
    h = rms_norm(x, w.ln2[i], eps)
    return x + swiglu(h @ w.gate_up[i].t()) @ w.down[i].t()
