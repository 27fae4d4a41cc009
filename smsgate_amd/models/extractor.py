"""The local structured-extraction LM (the MI355X replacement for the Gemini call).

Architecture: a Llama-family decoder with the exact shape of SmolLM2-135M —
hidden 576, 30 layers, 9 query / 3 key-value heads of 64, SwiGLU 1536,
RoPE θ = 1e5, RMSNorm ε = 1e-5, vocab 49 152, tied embeddings
(134.5 M parameters). It is small enough that one MI355X holds the weights
(270 MB bf16) plus thousands of KV slots in HBM, and it is the size class
that is fine-tuned for schema extraction in practice. No checkpoint exists on
the box, so weights are random-init (``init_std`` 0.02, HF default) unless a
safetensors file is given.

Weight layout is the serving layout (fused ``qkv`` [960, 576] and ``gate_up``
[3072, 576], ``[out, in]`` row-major) so the engine calls hipBLASLt once per
projection; :func:`reference_forward` is the plain PyTorch fp32/bf16 forward
used to validate the HIP path and for training.
"""
from __future__ import annotations

import dataclasses
import math
from dataclasses import asdict, dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

__all__ = ["ExtractorConfig", "CONFIGS", "ExtractorWeights", "reference_forward", "count_params", "span_config",
           "SPAN_PTR0", "qa_config"]


@dataclass(frozen=True)
class ExtractorConfig:
    name: str = "smollm-135m"
    vocab: int = 49152
    hidden: int = 576
    layers: int = 30
    heads: int = 9
    kv_heads: int = 3
    head_dim: int = 64
    inter: int = 1536
    rope_theta: float = 100000.0
    eps: float = 1e-5
    init_std: float = 0.02
    # > 0: the span-pointer answer format (serving/fsm.py build_span_fsm) -- embedding
    # rows ptr0 .. ptr0 + span_positions - 1 are the pointer tokens, and row ptr0 + j is
    # added to the input of prompt position j
    span_positions: int = 0
    # > 0: the one-forward span format (serving/qa.py): this many query tokens follow
    # ``body <ans>``; the span_positions pointer rows are as above, plus the end-pointer,
    # query, null and class rows of qa_layout
    qa_queries: int = 0

    @property
    def qkv_out(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def to_dict(self) -> dict:
        return asdict(self)


CONFIGS: Dict[str, ExtractorConfig] = {
    "smollm-135m": ExtractorConfig(),
    # same kernel-facing shapes family, small enough for CPU tests
    "tiny": ExtractorConfig(name="tiny", vocab=8192, hidden=128, layers=2, heads=4, kv_heads=2, head_dim=64,
                            inter=256),
    # fast-to-train working extractor (tests, small deployments): 5M params
    "small": ExtractorConfig(name="small", vocab=8192, hidden=256, layers=4, heads=4, kv_heads=2, head_dim=64,
                             inter=704),
    # larger variant (SmolLM2-360M shape) for capacity experiments
    "smollm-360m": ExtractorConfig(name="smollm-360m", hidden=960, layers=32, heads=15, kv_heads=5, head_dim=64,
                                   inter=2560),
}


# first pointer id of the span format: the tokenizer's 8 192 ids rounded to the lm_head tile
SPAN_PTR0 = 8192


def span_config(cfg: ExtractorConfig, positions: int = 130) -> ExtractorConfig:
    """``cfg`` for the span-pointer format: the embedding must hold the pointer rows
    (SmolLM2's 49 152 rows already do; the 8 192-row small models grow by 256)."""
    vocab = max(cfg.vocab, -(-(SPAN_PTR0 + positions) // 128) * 128)
    return dataclasses.replace(cfg, vocab=vocab, span_positions=positions)


def qa_config(cfg: ExtractorConfig, positions: int = 130, queries: int = 9) -> ExtractorConfig:
    """``cfg`` for the one-forward span format (serving/qa.py qa_layout)."""
    from ..serving.qa import qa_layout

    lay = qa_layout(SPAN_PTR0, positions, queries)
    return dataclasses.replace(cfg, vocab=max(cfg.vocab, lay.vocab), span_positions=positions, qa_queries=queries)


def count_params(cfg: ExtractorConfig) -> int:
    per = cfg.hidden * cfg.qkv_out + cfg.heads * cfg.head_dim * cfg.hidden + 3 * cfg.hidden * cfg.inter + 2 * cfg.hidden
    return cfg.vocab * cfg.hidden + cfg.layers * per + cfg.hidden


class ExtractorWeights(torch.nn.Module):
    """Parameters in serving layout. ``lm_head`` is tied to ``embed``."""

    def __init__(self, cfg: ExtractorConfig, device=None, dtype=torch.bfloat16, seed: Optional[int] = 0) -> None:
        super().__init__()
        self.cfg = cfg
        g = torch.Generator(device="cpu")
        if seed is not None:
            g.manual_seed(seed)

        def rnd(*shape):
            t = torch.empty(*shape, dtype=torch.float32)
            t.normal_(0.0, cfg.init_std, generator=g)
            return torch.nn.Parameter(t.to(dtype=dtype, device=device))

        def ones(n):
            return torch.nn.Parameter(torch.ones(n, dtype=dtype, device=device))

        H = cfg.hidden
        self.embed = rnd(cfg.vocab, H)
        self.qkv = torch.nn.ParameterList([rnd(cfg.qkv_out, H) for _ in range(cfg.layers)])
        self.o = torch.nn.ParameterList([rnd(H, cfg.heads * cfg.head_dim) for _ in range(cfg.layers)])
        self.gate_up = torch.nn.ParameterList([rnd(2 * cfg.inter, H) for _ in range(cfg.layers)])
        self.down = torch.nn.ParameterList([rnd(H, cfg.inter) for _ in range(cfg.layers)])
        self.ln1 = torch.nn.ParameterList([ones(H) for _ in range(cfg.layers)])
        self.ln2 = torch.nn.ParameterList([ones(H) for _ in range(cfg.layers)])
        self.ln_f = ones(H)

    @property
    def lm_head(self) -> torch.Tensor:
        return self.embed

    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        sd = {k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()}
        save_file(sd, path, metadata={k: str(v) for k, v in self.cfg.to_dict().items()})

    @classmethod
    def load(cls, path: str, cfg: ExtractorConfig, device=None, dtype=torch.bfloat16) -> "ExtractorWeights":
        from safetensors import safe_open
        from safetensors.torch import load_file

        with safe_open(path, framework="pt") as fh:  # the answer format is the checkpoint's own (metadata)
            meta = fh.metadata() or {}
        cfg = dataclasses.replace(cfg, vocab=int(meta.get("vocab", cfg.vocab)),
                                  span_positions=int(meta.get("span_positions", "0") or 0),
                                  qa_queries=int(meta.get("qa_queries", "0") or 0))
        w = cls(cfg, device="meta" if device is None else device, dtype=dtype, seed=None)
        sd = load_file(path, device=str(device) if device is not None else "cpu")
        w.load_state_dict({k: v.to(dtype) for k, v in sd.items()}, assign=True)
        return w


def _rope_tables(T: int, D: int, theta: float, device) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, device=device, dtype=torch.float32) / D))
    ang = torch.arange(T, device=device, dtype=torch.float32)[:, None] * inv[None, :]
    return ang.cos()[:, None, :], ang.sin()[:, None, :]  # [T, 1, D/2]


def _rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """rotate-half RoPE; ``x`` [..., T, H, D] with tables [T, 1, D/2]."""
    D = x.shape[-1]
    x1, x2 = x[..., : D // 2], x[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def _rms(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * w


def reference_forward(w: ExtractorWeights, ids: torch.Tensor, compute_dtype=torch.float32,
                      return_hidden: bool = False, add_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Full-sequence causal forward. ``ids``: [B, T] → logits [B, T, V] (fp32).

    Plain PyTorch (SDPA attention); differentiable, so it is also the training
    forward.  ``add_ids`` [B, T] (span format): a second embedding row added to each
    input (the position's pointer row; -1 = none).
    """
    cfg = w.cfg
    B, T = ids.shape
    x = F.embedding(ids, w.embed)
    if add_ids is not None:
        x = x + F.embedding(add_ids.clamp(min=0), w.embed) * (add_ids >= 0).unsqueeze(-1).to(x.dtype)
    x = x.to(compute_dtype)
    cos, sin = _rope_tables(T, cfg.head_dim, cfg.rope_theta, ids.device)  # once, not per layer
    for i in range(cfg.layers):
        h = _rms(x, w.ln1[i].to(compute_dtype), cfg.eps)
        qkv = h @ w.qkv[i].to(compute_dtype).t()
        q, k, v = qkv.split([cfg.heads * cfg.head_dim, cfg.kv_heads * cfg.head_dim, cfg.kv_heads * cfg.head_dim], -1)
        q = _rope(q.reshape(B, T, cfg.heads, cfg.head_dim), cos, sin).transpose(1, 2)
        k = _rope(k.reshape(B, T, cfg.kv_heads, cfg.head_dim), cos, sin).transpose(1, 2)
        v = v.reshape(B, T, cfg.kv_heads, cfg.head_dim).transpose(1, 2)
        # GQA inside SDPA: no repeat_interleave copies of K/V
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=1.0 / math.sqrt(cfg.head_dim),
                                           enable_gqa=cfg.heads != cfg.kv_heads)
        a = a.transpose(1, 2).reshape(B, T, cfg.heads * cfg.head_dim)
        x = x + a @ w.o[i].to(compute_dtype).t()
        h = _rms(x, w.ln2[i].to(compute_dtype), cfg.eps)
        g, u = (h @ w.gate_up[i].to(compute_dtype).t()).chunk(2, dim=-1)
        x = x + (F.silu(g) * u) @ w.down[i].to(compute_dtype).t()
    x = _rms(x, w.ln_f.to(compute_dtype), cfg.eps)
    if return_hidden:  # final-normed hidden states (training computes logits on answer rows only)
        return x
    return (x @ w.embed.to(compute_dtype).t()).float()
