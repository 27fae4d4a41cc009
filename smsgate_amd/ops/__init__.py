"""HIP/CDNA4 kernels of the local extractor LM, exposed to PyTorch.

The kernels live in ``csrc/llm_kernels.hip`` and are built in-tree for gfx950
(``smsgate_amd.ops.build``).  Each wrapper here validates shapes/dtypes on the
host *before* launching (a mis-shaped launch on the GPU box can fault the
device), then launches on ``torch.cuda.current_stream()`` — so the calls are
captured by ``torch.cuda.CUDAGraph``.

There is deliberately **no silent fallback**: on a GPU, a missing library is
an error (``SMSGATE_ALLOW_TORCH_OPS=1`` opts into the slow PyTorch reference
path, for debugging only).  The ``ref_*`` functions are the fp32 PyTorch
references the numerics tests compare against.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np
import torch

from . import build as _build

__all__ = [
    "load_library",
    "have_kernels",
    "rmsnorm_residual",
    "silu_mul",
    "rope_qkv_cache",
    "kv_copy_prefix",
    "attn_prefill",
    "attn_decode",
    "fsm_sample",
    "spec_plan",
    "attn_spec",
    "spec_verify",
    "spec_verify_keys",
    "fsm_commit",
    "gemm_argmax",
    "copy_masks",
    "qa_decode",
    "qa_params",
    "embed_rows_add_ids",
    "ref_copy_masks",
    "SPEC_MAX_K",
    "gemm",
    "gemm_cfg",
    "gemm_qkv_rope",
    "interleave_gate_up",
    "fold_norm",
    "rope_table",
    "vt_shape",
    "vt_to_rows",
    "rows_to_vt",
    "ref_rmsnorm",
    "ref_silu_mul",
    "ref_rope",
    "ref_attention",
    "ref_gemm",
]

_lib: Optional[ctypes.CDLL] = None
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_vp = ctypes.c_void_p
_ip = ctypes.c_void_p  # int32 device pointers travel as void*


def _declare(lib: ctypes.CDLL) -> None:
    lib.sg_rmsnorm_residual.argtypes = [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_float, _vp]
    lib.sg_silu_mul.argtypes = [_vp, _vp, _c_int, _c_int, _vp]
    lib.sg_rope_qkv_cache.argtypes = [_vp, _ip, _ip, _vp, _vp, _vp, _vp] + [_c_int] * 6 + [_vp]
    lib.sg_kv_copy_prefix.argtypes = [_vp, _vp, _ip] + [_c_int] * 6 + [_vp]
    lib.sg_attn_prefill.argtypes = [_vp, _ip, _ip, _ip, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp,
                                    _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp]
    lib.sg_attn_decode.argtypes = [_vp, _ip, _ip, _ip, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp,
                                   _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp]
    lib.sg_attn_decode_valu.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_valu.restype = _c_int
    lib.sg_attn_decode_v1.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_v1.restype = _c_int
    lib.sg_attn_decode_cascade.argtypes = lib.sg_attn_decode.argtypes[:-1] + [_vp, _vp, _vp]
    lib.sg_attn_decode_grouped.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_grouped.restype = _c_int
    lib.sg_attn_decode_grouped6.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_grouped6.restype = _c_int
    lib.sg_attn_decode_grouped_h.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_grouped_h.restype = _c_int
    lib.sg_attn_decode_grouped_pf.argtypes = lib.sg_attn_decode.argtypes
    lib.sg_attn_decode_grouped_pf.restype = _c_int
    lib.sg_attn_decode_split.argtypes = lib.sg_attn_decode.argtypes[:-1] + [_c_int, _vp]
    lib.sg_attn_spec.argtypes = [_vp, _ip, _ip, _ip, _ip, _ip, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp, _c_int,
                                 _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _vp]
    lib.sg_attn_spec.restype = _c_int
    lib.sg_attn_decode_split.restype = _c_int
    lib.sg_attn_decode_cascade.restype = _c_int
    lib.sg_fsm_sample.argtypes = [_vp, _c_int, _vp, _ip, _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _c_int,
                                  _ip, _ip, _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _c_int, _c_float,
                                  ctypes.c_uint, _ip, _vp, _vp]
    lib.sg_gemm.argtypes = [_vp, _c_int, _vp, _vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                            _c_float, _c_int, _vp, _vp, _c_int, _vp]
    lib.sg_gemm_qkv_rope.argtypes = [_vp, _c_int, _vp, _c_int, _c_int, _c_float, _c_int, _ip, _ip, _vp, _vp, _vp,
                                     _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _vp]
    lib.sg_prefill_forward.argtypes = [_c_int] + [_vp] * 8 + [_vp] + [_c_int] * 9 + [_ip, _ip, _vp, _c_int, _ip, _ip,
                                                                               _ip, _c_int, _c_int, _c_float, _vp,
                                                                               _vp, _vp, _vp, _c_int, _c_float] + \
        [_c_int] * 4 + [_vp]
    lib.sg_prefill_forward.restype = _c_int
    lib.sg_embed_rows.argtypes = [_ip, _vp, _vp, _c_int, _c_int, _c_int, _vp]
    lib.sg_embed_rows.restype = _c_int
    lib.sg_embed_rows_add.argtypes = [_ip, _ip, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp]
    lib.sg_embed_rows_add.restype = _c_int
    lib.sg_sparse_argmax.argtypes = [_vp, _ip, _c_int, _c_int, _ip, _vp, _vp, _c_int, _vp, _c_int, _c_float,
                                     _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _c_int, _c_int, _vp, _vp]
    lib.sg_sparse_argmax.restype = _c_int
    lib.sg_gemm_probe.argtypes = [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp]
    lib.sg_gemm_probe.restype = _c_int
    lib.sg_gemm_set_group_m.argtypes = [_c_int]
    lib.sg_gemm_set_group_m.restype = None
    lib.sg_set_prefill_impl.argtypes = [_c_int]
    lib.sg_set_prefill_impl.restype = None
    lib.sg_set_attn_merge.argtypes = [_c_int]
    lib.sg_set_attn_merge.restype = None
    lib.sg_set_prefill_split.argtypes = [_c_int]
    lib.sg_set_prefill_split.restype = None
    fsm_t = [_vp, _ip, _ip, _ip, _ip, _ip, _c_int]  # masks, state_mask, next_sep, next_tok, enum_tok, enum_next, E
    lib.sg_spec_plan.argtypes = fsm_t + [_c_int, _c_int, _ip, _ip] + [_c_int] * 5 + [_ip] * 6 + [_c_int] + \
        [_ip, _ip, _c_int, _vp, _ip, _c_int] + [_ip] * 8 + [_vp]
    lib.sg_spec_plan.restype = _c_int
    lib.sg_spec_verify.argtypes = [_vp, _c_int, _vp, _ip, _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _c_int,
                                   _ip, _ip, _ip, _ip, _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _c_int, _ip, _vp, _vp]
    lib.sg_spec_verify.restype = _c_int
    lib.sg_spec_verify_keys.argtypes = [_vp] + fsm_t + [_c_int] * 3 + [_ip] * 10 + [_c_int, _c_int, _vp, _vp]
    lib.sg_spec_verify_keys.restype = _c_int
    lib.sg_fsm_commit.argtypes = [_vp, _ip] + fsm_t + [_c_int] * 3 + [_ip] * 6 + [_c_int, _c_int, _vp]
    lib.sg_fsm_commit.restype = _c_int
    lib.sg_span_commit.argtypes = [_vp, _ip] + fsm_t + [_c_int] * 3 + [_ip] * 4 + [_c_int, _c_int] + [_ip] * 6 + \
        [_c_int, _c_int, _vp]
    lib.sg_span_commit.restype = _c_int
    lib.sg_gemm_argmax.argtypes = [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_float, _c_int, _c_int, _ip, _ip, _vp,
                                   _vp, _vp, _c_int, _ip, _vp, _vp]
    lib.sg_gemm_argmax.restype = _c_int
    lib.sg_copy_masks.argtypes = [_vp, _ip, _c_int, _c_int, _ip, _vp, _ip, _ip, _ip, _ip, _ip, _c_int, _c_int, _vp,
                                  _vp]
    lib.sg_copy_masks.restype = _c_int
    lib.sg_qa_decode.argtypes = [_vp, _vp, _c_int, _vp, _c_int, _c_float, _ip, _ip, _vp, _c_int, _ip, _ip, _vp, _vp,
                                 _vp, _c_int, _c_int, _vp]
    lib.sg_qa_decode.restype = _c_int
    lib.sg_qa_params_size.argtypes = []
    lib.sg_qa_params_size.restype = _c_int
    lib.sg_embed_rows_add_ids.argtypes = [_ip, _ip, _vp, _vp, _c_int, _c_int, _c_int, _vp]
    lib.sg_embed_rows_add_ids.restype = _c_int
    # training step (csrc/train_kernels.hip, models/train_ops.py)
    lib.sg_rms_fwd.argtypes = [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_float, _vp]
    lib.sg_rms_bwd.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp]
    lib.sg_rope_split.argtypes = [_c_int, _vp, _vp, _vp, _vp, _vp, _vp] + [_c_int] * 6 + [_vp]
    lib.sg_swiglu_fwd.argtypes = [_vp, _vp, _c_int, _c_int, _vp]
    lib.sg_swiglu_bwd.argtypes = [_vp, _vp, _vp, _c_int, _c_int, _vp]
    lib.sg_attn_train_fwd.argtypes = [_vp] * 5 + [_c_int] * 4 + [_c_float, _vp]
    lib.sg_attn_train_bwd.argtypes = [_vp] * 10 + [_c_int] * 4 + [_c_float, _vp]
    for fn in (lib.sg_rms_fwd, lib.sg_rms_bwd, lib.sg_rope_split, lib.sg_swiglu_fwd, lib.sg_swiglu_bwd,
               lib.sg_attn_train_fwd, lib.sg_attn_train_bwd):
        fn.restype = _c_int
    for f in ("sg_gemm", "sg_gemm_qkv_rope", "sg_rmsnorm_residual", "sg_silu_mul", "sg_rope_qkv_cache", "sg_attn_prefill", "sg_attn_decode",
              "sg_fsm_sample", "sg_version", "sg_kv_copy_prefix"):
        getattr(lib, f).restype = _c_int


def load_library(build_if_missing: bool = True) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    path = _build.LIB
    if build_if_missing and _build.needs_build():
        _build.build()
    if not path.exists():
        raise RuntimeError(f"HIP kernel library missing: {path} (run python -m smsgate_amd.ops.build)")
    lib = ctypes.CDLL(str(path))
    _declare(lib)
    _lib = lib
    return lib


def have_kernels() -> bool:
    try:
        load_library()
        return True
    except Exception:
        return False


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name} failed (rc={rc})")


def _req(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")


# ---------------------------------------------------------------------------- ops
def rmsnorm_residual(residual: torch.Tensor, weight: torch.Tensor, eps: float,
                     x: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``residual += x`` (in place, if given); returns ``rmsnorm(residual) * weight``."""
    T, H = residual.shape
    _req(residual, torch.bfloat16, "residual")
    _req(weight, torch.bfloat16, "weight")
    if x is not None:
        _req(x, torch.bfloat16, "x")
        assert x.shape == residual.shape
    if out is None:
        out = torch.empty_like(residual)
    assert weight.numel() == H and out.shape == residual.shape
    _check(load_library().sg_rmsnorm_residual(_p(x), _p(residual), _p(weight), _p(out), T, H, eps, _stream()),
           "rmsnorm_residual")
    return out


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    T, I2 = gu.shape
    _req(gu, torch.bfloat16, "gu")
    I = I2 // 2
    if out is None:
        out = gu.new_empty((T, I))
    assert out.shape == (T, I)
    _check(load_library().sg_silu_mul(_p(gu), _p(out), T, I, _stream()), "silu_mul")
    return out


GEMM_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (128, 64), 5: (64, 64), 6: (64, 64),
              7: (128, 128), 8: (64, 128), 9: (256, 128), 10: (256, 256), 11: (128, 256), 12: (256, 64),
              13: (128, 128), 14: (256, 128), 15: (128, 256), 16: (256, 64), 17: (32, 64), 18: (32, 64),
              19: (256, 256), 20: (256, 256), 21: (128, 96), 22: (64, 96), 23: (128, 192), 24: (256, 96),
              25: (128, 96), 26: (64, 192), 27: (32, 96), 28: (128, 192), 29: (256, 96),
              30: (128, 96), 31: (64, 96), 32: (256, 192), 33: (128, 192), 34: (256, 192),
              35: (256, 192), 36: (256, 192), 37: (256, 192), 38: (256, 192), 42: (256, 256)}
# cfg -> (BM, BN); 4..8 are 3/4-stage pipelines, 9..16 are 8-wave blocks (14..16: 3/4 stages),
# 17/18: 32-row tiles (2 / 4 stages) for small decode buckets
# a 256x256 plain-output tile does not fit the LDS staging; 19 is the staggered 8-wave
# SwiGLU kernel (gemm256_swiglu_kernel), 20 its persistent form, 42 = 20 with both A register
# sets (A/B)
GEMM_SWIGLU_ONLY = {10, 19, 20, 42}
# 21..26: 48-wide wave tiles (96 / 192-wide blocks) for the N = 576 residual GEMMs: no SwiGLU
# 28 / 29: 128x192 / 256x96 with 4 waves (64x96 wave tiles); 30 / 31: 128x96 / 64x96 with 8 waves
# 32: 256x192 with 8 waves (64x96 wave tiles); 33 / 34: 128x192 / 256x192 with BK 32 and 4 stages
GEMM_NO_SWIGLU = {21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38}
# 35..38: the persistent, staggered 256x192 residual GEMM (gemm256p_resid_kernel: 4 / 5
# ring buffers, 16x16x32 / 32x32x16 MFMAs) -- epi "resid" only
GEMM_RESID_ONLY = {35, 36, 37, 38}
_EPI = {"store": 0, "resid": 1, "swiglu": 2}


GEMM_MIN_TILES = int(os.environ.get("SMSGATE_GEMM_MIN_TILES", "480"))
# M at or below which the 32-row tile (cfg 17) competes in gemm_cfg; 0 = never
GEMM_SMALL_M = int(os.environ.get("SMSGATE_GEMM_SMALL_M", "1024"))


# Measured exceptions to the tile rule below (scripts/gemm_tune.py, interleaved rounds,
# profiles/r02_gemm_tune.json), keyed by (epilogue, N, K): [(M_lo, M_hi, cfg)].
#   SwiGLU gate/up 3072x576: 256x256 8-wave tiles at 4608 rows (26.7 vs 28.4 us) and at
#     prefill halves of 16384 (73.9 vs 80.3 us); 128x128 stays best at 9216 (47.5 vs 49.4).
#   o-proj 576x576 + residual: 64x64 tiles at 9216 rows (14.3 vs 15.9 us) (re-confirmed below).
# End to end the bench is unchanged within noise (27 571 vs 27 491 msgs/s, three
# interleaved runs each, profiles/r02_gemm_measured_ab.jsonl).
#   SwiGLU gate/up with the staggered 256x256 kernel (cfg 19, scripts/gemm256_check.py,
#     producer row partials): 22.2 / 41.6 / 67.2 us at 4608 / 9216 / 16384 rows vs 24.1 /
#     43.8 / 68.2 for the best of cfg 0 and 10; its persistent form (cfg 20, the default
#     from 4096 rows) 39.1 / 60.9 us at 9216 / 16384 (profiles/r02_gemm256_check.json).
#   Re-swept with the engine's norm flavour (producer partials in / out; interleaved,
#   profiles/r02s3_gemm_tune.json): gate/up at 2304 rows 128x128 8-wave (13.7 vs 16.9 us),
#   at 4608 rows (one tile round: nothing for persistence to overlap) cfg 19 (21.1 vs 21.6);
#   o-proj at 9216 rows 64x64 (14.7 vs 16.4 us).
#   Round 3: 96-wide tiles (48-wide wave tiles: 6 B of LDS reads per output instead of 8
#   for 64x64 / 32x32 wave tiles) for the N = 576 residual GEMMs, interleaved with every
#   older config at the engine's flavour (profiles/r03_gemm96_tune.json): down-proj 128x96
#   25.0 / 40.3 us at 9216 / 16384 rows vs 28.2 / 43.4 (128x64), 64x96 15.8 vs 18.5 at
#   4608; o-proj 64x96 8.3 / 20.3 us at 4608 / 16384 vs 8.8 / 22.4, 128x96 13.0 vs 14.9
#   (64x64) at 9216.  Both residual GEMMs keep BN = 96 at EVERY row count (32x96 below
#   2048 rows): the producer-norm partials then always come as the same 6 parts summed in
#   the same order, so a row's result does not depend on the batch it runs in (split vs
#   single prefill, spec vs plain decode: tests/test_engine_gpu.py, test_spec_gpu.py).
#   The price below 2048 rows: 32x96 runs 5-25 % behind 32x64 (down-proj 9.3 vs 7.7 us at
#   256 rows, 9.7 vs 8.4 at 1024; profiles/r03_resid_small_m_tune.json) -- small decode
#   buckets only, i.e. serving latency at low load, not the throughput bench's 9216-row
#   halves.
#   Round 5 (the qa engine's one-forward batches: 110 k / 220 k prefill rows), interleaved
#   at 55 296 / 110 592 rows (profiles/r05_gemm_tune_qa.json): 128x192 with 4 waves
#   (64x96 wave tiles, cfg 28) beats the 96-wide tiles for both residual GEMMs -- down-proj
#   116.0 / 233.4 us vs 121.6 / 270.0 (cfg 21), o-proj 59.4 / 105.2 vs 59.6 / 117.8 (cfg
#   22) -- and the QKV+RoPE GEMM (qkv_cfg).  Its x² parts stay 96 columns wide (two per
#   tile, each summed like a 96-wide tile's), so results do not depend on the config.
#   With both fitting 256 registers (r05_gemm_tune_resid_u.json, 3 interleaved rounds):
#   down-proj at 27 648 rows 59.7 us on 28 vs 67.6 on 21, so 28 from 16 384 rows; the
#   256x192 8-wave tile (cfg 32) trails 28 at every size (257.8 vs 223.5 us at 110 592).
GEMM_MEASURED = {
    ("swiglu", 3072, 576): [(2048, 4095, 13), (4096, 6143, 19), (6144, 1 << 30, 20)],
    ("resid", 576, 576): [(1, 2047, 27), (2048, 6143, 22), (6144, 12287, 21), (12288, 32767, 22),
                          (32768, 1 << 30, 28)],
    ("resid", 576, 1536): [(1, 2047, 27), (2048, 6143, 22), (6144, 16383, 21), (16384, 1 << 30, 28)],
} if os.environ.get("SMSGATE_GEMM_MEASURED", "1") != "0" else {}


def gemm_cfg(M: int, N: int, min_tiles: Optional[int] = None, epi: Optional[str] = None,
              K: Optional[int] = None) -> int:
    """Tile config for an M×N output: a measured exception for (``epi``, N, ``K``) at this
    M (:data:`GEMM_MEASURED`), else the biggest tile that still gives ≳2 blocks per CU
    (256 CUs), else the config with the most blocks (the 32-row tile only for M <=
    ``GEMM_SMALL_M``)."""
    for lo, hi, c in GEMM_MEASURED.get((epi, N, K), ()):
        if lo <= M <= hi:
            return c
    min_tiles = GEMM_MIN_TILES if min_tiles is None else min_tiles
    best, best_tiles = -1, -1
    # the 4-wave configs; 8-wave ones and the 4-stage 32-row tile are explicit opt-ins
    for cfg in list(range(9)) + ([17] if M <= GEMM_SMALL_M else []):
        bm, bn = GEMM_TILES[cfg]
        if N % bn:
            continue
        tiles = -(-M // bm) * (N // bn)
        if tiles >= min_tiles:
            return cfg
        if tiles > best_tiles:
            best, best_tiles = cfg, tiles
    if best < 0:
        raise ValueError(f"gemm: N={N} is not a multiple of 64")
    return best


def gemm_set_group_m(gm: int) -> None:
    """Tile rasterisation of the fused GEMMs: M-tiles per group (1 = row-major)."""
    load_library().sg_gemm_set_group_m(int(gm))


SS_PARTS = 16  # csrc/gemm_kernels.hip: x² partials per row (producer N tiles, zero-padded)


def ss_buffer(M: int, device) -> torch.Tensor:
    """Zeroed fp32 ``[SS_PARTS, M]`` row-partials image for ``gemm(ss_out=..)`` / ``ss_in``
    (part-major: column ``m`` holds row ``m``'s partials)."""
    return torch.zeros(SS_PARTS, (M + 3) // 4 * 4, dtype=torch.float32, device=device)  # 16-B row groups


def _ss_check(ss: Optional[torch.Tensor], M: int, name: str) -> int:
    """Validates a row-partials image; returns its row capacity (0 for None)."""
    if ss is None:
        return 0
    if ss.dtype != torch.float32 or ss.dim() != 2 or ss.stride(1) != 1 or ss.shape[0] != SS_PARTS \
            or ss.shape[1] < M or not ss.is_cuda:
        raise ValueError(f"{name}: fp32 [{SS_PARTS}, >= {M}] row partials required (ops.ss_buffer)")
    return ss.stride(0)


def gemm(a: torch.Tensor, w: torch.Tensor, *, epi: str = "store", norm_eps: Optional[float] = None,
         resid: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
         cfg: Optional[int] = None, ss_in: Optional[torch.Tensor] = None,
         ss_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused MFMA GEMM ``out = EPI(rowscale ⊙ (a @ w.T))`` (csrc/gemm_kernels.hip).

    ``a`` [M, K] (row stride may exceed K), ``w`` [N, K] bf16.  ``norm_eps``: apply
    RMSNorm to the rows of ``a`` (the norm weight must already be folded into
    ``w`` — :func:`fold_norm`).  ``epi``: ``store``; ``resid`` (``out = resid +
    result``; ``out`` defaults to ``resid`` itself, updated in place); ``swiglu``
    (``w`` rows interleaved by :func:`interleave_gate_up`, output N/2 wide).

    ``ss_out`` (``epi='resid'`` only, :func:`ss_buffer`): receives, per N tile, the
    sum of squares of each output row (as stored, bf16) — the next RMSNorm GEMM's
    row scales; its other columns must stay zero.  ``ss_in`` (with ``norm_eps``):
    such a buffer for the rows of ``a``; the GEMM sums its partials instead of
    accumulating x² itself."""
    M, K = a.shape
    N = w.shape[0]
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("gemm: bf16 operands required")
    if a.stride(1) != 1 or not w.is_contiguous() or w.shape[1] != K or not a.is_cuda:
        raise ValueError(f"gemm: bad operands a{tuple(a.shape)}/{a.stride()} w{tuple(w.shape)}")
    if K % 64 or N % 64 or a.stride(0) % 8:
        raise ValueError(f"gemm: K={K} and N={N} must be multiples of 64")
    e = _EPI[epi]
    n_out = N // 2 if e == 2 else N
    if e == 1:
        if resid is None or resid.shape != (M, n_out) or resid.dtype != torch.bfloat16 or resid.stride(1) != 1:
            raise ValueError("gemm: epi='resid' needs a bf16 [M, N] residual")
        if out is None:
            out = resid
    if out is None:
        out = a.new_empty((M, n_out))
    if out.shape != (M, n_out) or out.stride(1) != 1 or out.stride(0) % 8 or out.dtype != torch.bfloat16:
        raise ValueError("gemm: bad output")
    if M == 0:
        return out
    c = gemm_cfg(M, N, epi=epi, K=K) if cfg is None else cfg
    if ss_in is not None and norm_eps is None:
        raise ValueError("gemm: ss_in needs norm_eps")
    ld_in = _ss_check(ss_in, M, "gemm ss_in")
    ld = _ss_check(ss_out, M, "gemm ss_out") or ld_in
    if ss_out is not None and (e != 1 or N // GEMM_TILES[c][1] > SS_PARTS):
        raise ValueError(f"gemm: ss_out needs epi='resid' and at most {SS_PARTS} N tiles")
    if ss_in is not None and ss_out is not None and ld_in != ld:
        raise ValueError("gemm: ss_in / ss_out row strides differ")
    norm = 0 if norm_eps is None else (2 if ss_in is not None else 1)
    rc = load_library().sg_gemm(_p(a), a.stride(0), _p(w), _p(out), out.stride(0), _p(resid),
                                0 if resid is None else resid.stride(0), M, N, K, e, norm,
                                float(norm_eps or 0.0), c, _p(ss_in), _p(ss_out), ld, _stream())
    _check(rc, "gemm")
    return out


def qkv_cfg(M: int, nh: int = 9, nkv: int = 3) -> int:
    """Tile config of the QKV+RoPE GEMM at M rows.  64x64 tiles: the V^T scatter of the
    epilogue favours more, smaller tiles (kbench, B=4096/8192: 17.8/27.6 us vs 22.0/31.3
    us with 128x64); 32-row tiles up to 2048 rows (7.4 / 8.2 / 11.4 vs 10.1 / 10.7 / 12.3
    us at 512 / 1024 / 2048, profiles/r01c_kbench_small_buckets.json); 128x192 with 4
    waves (64x96 wave tiles) at the 9 216-row decode halves (24.45 vs 25.10 us,
    profiles/r03s2_tiles_tune.json); 128x64 from 12 288 rows (prefill halves: 39.0 vs 40.7
    us at 16 384, r02s3_gemm_tune.json); 128x192 again from 32 768 rows (the qa engine's
    batches: 113.8-114.5 / 222.1 vs 133.7 / 264.4 us at 55 296 / 110 592 rows,
    profiles/r05_gemm_tune_qa.json).  Every config accumulates each output in the
    same K order, so the choice never changes a result.  192-wide tiles hold three
    heads: only for head counts divisible by 3."""
    three = nh % 3 == 0 and nkv % 3 == 0
    if M <= 2 * GEMM_SMALL_M:
        return 17
    if M >= 32768 and three:  # the qa engine's batches: 222 vs 264 us at 110 592 rows (r05_gemm_tune_qa.json)
        return 28
    if M >= 12288:
        return 1
    return 28 if M >= 6144 and three else 3


def gemm_qkv_rope(x: torch.Tensor, w: torch.Tensor, eps: float, pos: torch.Tensor, slot: torch.Tensor,
                  cos_sin: torch.Tensor, q_out: torch.Tensor, k_cache: torch.Tensor, vt_cache: torch.Tensor,
                  nh: int, nkv: int, p0: int, cfg: Optional[int] = None,
                  ss_in: Optional[torch.Tensor] = None) -> None:
    """``rope(rmsnorm(x) @ w.T)`` scattered into ``q_out`` and the KV cache (one fused
    kernel; ``w`` has the norm weight folded in).  Same result as :func:`gemm` +
    :func:`rope_qkv_cache`."""
    M, K = x.shape
    S, nkv_, Lmax, D = k_cache.shape
    if x.dtype != torch.bfloat16 or x.stride(1) != 1 or x.stride(0) % 8 or K % 64:
        raise ValueError("gemm_qkv_rope: bad activation")
    if w.shape != ((nh + 2 * nkv) * 64, K) or not w.is_contiguous() or D != 64 or nkv_ != nkv:
        raise ValueError("gemm_qkv_rope: bad weight / cache")
    _req(pos, torch.int32, "pos")
    _req(slot, torch.int32, "slot")
    _req(cos_sin, torch.float32, "cos_sin")
    assert vt_cache.shape == vt_shape(S, nkv, D, Lmax) and pos.numel() >= M and slot.numel() >= M
    assert q_out.is_contiguous() and q_out.numel() >= M * nh * D and q_out.dtype == torch.bfloat16
    if M == 0:
        return
    if cfg is None:
        cfg = qkv_cfg(M, nh, nkv)
    ld = _ss_check(ss_in, M, "gemm_qkv_rope ss_in")
    rc = load_library().sg_gemm_qkv_rope(_p(x), x.stride(0), _p(w), M, K, float(eps), cfg, _p(pos), _p(slot),
                                         _p(cos_sin), _p(q_out), _p(k_cache), _p(vt_cache), nh, nkv, Lmax, p0,
                                         _p(ss_in), ld, _stream())
    _check(rc, "gemm_qkv_rope")


class LayerPointers:
    """Per-layer device addresses of a fused serving model (int64 host arrays) for the
    native launch sequences (``csrc/runtime.hip``): weights, KV caches, shared prefix.
    The tensors must stay alive (and in place) as long as this object is used."""

    def __init__(self, w_qkv, w_o, w_gu, w_down, k_cache, vt_cache, pk, pvt):
        def arr(ts):
            return np.asarray([t.data_ptr() for t in ts], dtype=np.int64)

        L = len(w_qkv)
        self.L = L
        self.arrays = [arr(w_qkv), arr(w_o), arr(w_gu), arr(w_down), arr(k_cache[i] for i in range(L)),
                       arr(vt_cache[i] for i in range(L)), arr(pk[i] for i in range(L)), arr(pvt[i] for i in range(L))]
        self.ptrs = [a.ctypes.data for a in self.arrays]


def prefill_forward(lp: LayerPointers, x: torch.Tensor, *, H: int, I: int, nh: int, nkv: int, D: int, Lmax: int,
                    P0: int, P0pad: int, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor, p0: int,
                    cu_q: torch.Tensor, q_start: torch.Tensor, seq_slot: torch.Tensor, max_q: int, scale: float,
                    q: torch.Tensor, a: torch.Tensor, act: torch.Tensor, ss: Optional[torch.Tensor], eps: float,
                    layers: Optional[int] = None) -> None:
    """The fused prefill forward (every layer -- or the first ``layers`` -- : QKV+RoPE+KV write, varlen prefill
    attention, o-proj + residual, SwiGLU gate/up, down-proj + residual) as ONE native
    call (``sg_prefill_forward``) — the kernels and tile configs of ``gemm_qkv_rope`` /
    ``attn_prefill`` / ``gemm`` launched from C instead of ~150 Python wrapper calls.
    ``x`` [T, H] is the residual stream (updated in place); ``q``/``a``/``act`` scratch."""
    T = x.shape[0]
    if T == 0:
        return
    assert x.is_contiguous() and x.shape[1] == H and q.numel() >= T * nh * D and a.numel() >= T * nh * D
    assert act.is_contiguous() and act.shape[1] == I and act.shape[0] >= T
    nseq = cu_q.numel() - 1
    cfg_qkv = qkv_cfg(T, nh, nkv)  # gemm_qkv_rope's rule
    cfg_o = gemm_cfg(T, H, epi="resid", K=nh * D)
    cfg_gu = gemm_cfg(T, 2 * I, epi="swiglu", K=H)
    cfg_down = gemm_cfg(T, H, epi="resid", K=I)
    ld = _ss_check(ss, T, "prefill_forward ss")
    L = lp.L if layers is None else int(layers)
    if not 0 <= L <= lp.L:
        raise ValueError(f"prefill_forward: {L} layers of {lp.L}")
    rc = load_library().sg_prefill_forward(
        L, *lp.ptrs, _p(x), T, H, I, nh, nkv, D, Lmax, P0, P0pad, _p(pos), _p(slot), _p(cos_sin), p0, _p(cu_q),
        _p(q_start), _p(seq_slot), nseq, max_q, float(scale), _p(q), _p(a), _p(act), _p(ss), ld, float(eps),
        cfg_qkv, cfg_o, cfg_gu, cfg_down, _stream())
    _check(rc, "prefill_forward")


def fold_norm(w: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
    """``W' = W · diag(norm_w)`` so that ``rmsnorm(x)·norm_w @ W.T == rowscale(x) ⊙ (x @ W'.T)``."""
    return (w.float() * norm_w.float()[None, :]).to(w.dtype).contiguous()


def interleave_gate_up(gate_up: torch.Tensor, group: int = 16) -> torch.Tensor:
    """[2I, K] (gate rows then up rows) → rows interleaved in groups of 16 (g0..15, u0..15, g16..)."""
    two_i, K = gate_up.shape
    i = two_i // 2
    g, u = gate_up[:i].reshape(i // group, group, K), gate_up[i:].reshape(i // group, group, K)
    return torch.stack([g, u], dim=1).reshape(two_i, K).contiguous()


def rope_table(max_pos: int, head_dim: int, theta: float, device) -> torch.Tensor:
    """``[max_pos, head_dim/2, 2]`` fp32 (cos, sin) — computed once on the host side (Appendix B)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], dim=-1).to(torch.float32).contiguous().to(device)


def rope_qkv_cache(qkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
                   q_out: torch.Tensor, k_cache: torch.Tensor, vt_cache: torch.Tensor,
                   nh: int, nkv: int, head_dim: int, p0: int) -> None:
    T = qkv.shape[0]
    _req(qkv, torch.bfloat16, "qkv")
    _req(pos, torch.int32, "pos")
    _req(slot, torch.int32, "slot")
    _req(cos_sin, torch.float32, "cos_sin")
    S, nkv_, Lmax, D = k_cache.shape
    assert qkv.shape[1] == (nh + 2 * nkv) * head_dim and D == head_dim and nkv_ == nkv
    assert vt_cache.shape == vt_shape(S, nkv, D, Lmax), (vt_cache.shape, vt_shape(S, nkv, D, Lmax))
    assert q_out.shape[0] >= T and q_out.numel() >= T * nh * D
    assert pos.numel() == T and slot.numel() == T
    _check(load_library().sg_rope_qkv_cache(_p(qkv), _p(pos), _p(slot), _p(cos_sin), _p(q_out), _p(k_cache),
                                            _p(vt_cache), T, nh, nkv, D, Lmax, p0, _stream()), "rope_qkv_cache")


def set_prefill_impl(impl: str) -> None:
    """``"auto"`` (default: ``st32``; past 16 query heads per KV head ``per_head`` up
    to 384 sequences per launch, ``gqa`` above), ``"gqa"`` (one wave per KV head, K/V loaded once per GQA group,
    prefetched), ``"per_head"`` (one wave per query head: G x the waves, which
    fills the chip better at small batches; ``profiles/r01c_prefill_key_split_ab.txt``)
    or ``"multi"`` (per head, every K/V tile of a 3-tile chunk loaded at once), or
    ``"st"`` / ``"st32"`` / ``"st64"`` (transposed register formulation, S^T = K·Q^T and
    O^T = V^T·P^T: one wave per 16 / 32 / 64 (query, head) columns of one KV head,
    P never leaves registers)."""
    load_library().sg_set_prefill_impl({"gqa": 0, "per_head": 1, "auto": 2, "multi": 3, "st": 4, "st32": 5, "st64": 6, "st32pf": 7, "stpf": 8, "st64pf": 9}[impl])


def set_attn_merge(on: bool) -> None:
    """``True`` (default): the transposed attention kernels (verify, grouped decode,
    prefill ``st``/``st32``) walk the shared prefix and a row's own keys as ONE
    stream of 32-key tiles when ``P0 % 4 == 0`` (ceil((P0 + own) / 32) tiles instead
    of ceil(P0 / 32) + ceil(own / 32)); ``False``: prefix tiles, then own tiles."""
    load_library().sg_set_attn_merge(1 if on else 0)


def set_prefill_split(ks: int) -> None:
    """Key split of the GQA prefill kernel: 1 = one wave per (16-query tile,
    sequence, KV head); 2 = two waves deal its key tiles and merge in LDS."""
    if ks not in (1, 2):
        raise ValueError("prefill key split must be 1 or 2")
    load_library().sg_set_prefill_split(ks)


def attn_prefill(q: torch.Tensor, cu_q: torch.Tensor, q_start: torch.Tensor, slot: torch.Tensor, max_q: int,
                 k_cache: torch.Tensor, vt_cache: torch.Tensor, pk: torch.Tensor, pvt: torch.Tensor, P0: int,
                 out: torch.Tensor, scale: float) -> torch.Tensor:
    """Causal varlen attention. ``q``: [T, nh, D]; sequence ``b`` owns rows
    ``cu_q[b]:cu_q[b+1]`` whose own offsets start at ``q_start[b]``; keys are the
    shared prefix (``pk``/``pvt``, ``P0`` valid of ``P0pad``) followed by the slot's own keys."""
    T, nh, D = q.shape
    S, nkv, Lmax, _ = k_cache.shape
    P0pad = pk.shape[1]
    nseq = cu_q.numel() - 1
    assert pk.shape == (nkv, P0pad, D) and pvt.shape == vt_shape(1, nkv, D, P0pad)[1:]
    assert vt_cache.shape == vt_shape(S, nkv, D, Lmax)
    assert slot.numel() == nseq and q_start.numel() == nseq and P0 <= P0pad
    _check(load_library().sg_attn_prefill(_p(q), _p(cu_q), _p(q_start), _p(slot), _p(k_cache), _p(vt_cache),
                                          _p(pk), _p(pvt), P0, P0pad, _p(out), nseq, max_q, nh, nkv, D, Lmax,
                                          scale, _stream()), "attn_prefill")
    return out


def attn_decode(q: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, k_cache: torch.Tensor,
                vt_cache: torch.Tensor, pk: torch.Tensor, pvt: torch.Tensor, P0: int, out: torch.Tensor,
                scale: float, done: Optional[torch.Tensor] = None, impl: str = "cascade",
                scratch: Optional[tuple] = None) -> torch.Tensor:
    """One query token per row; rows with ``done[b] != 0`` are skipped (output untouched).

    ``impl="cascade"`` (default): shared-prefix pass over 16 query rows per wave +
    own-key pass seeded with the exact prefix softmax state; ``scratch`` =
    ``(pre_o [>=B, nh, D] fp32, pre_lse [>=B, nh] fp32)`` (allocated if omitted).
    ``"grouped"``: 16/G sequences per wave, the shared prefix multiplied once for
    all of them, then each sequence's own keys with per-column masks (no scratch);
    ``"grouped_pf"``: the same with the next key tile's loads issued before the
    current tile's MFMAs (one flattened tile stream per wave); ``"grouped6"``: the
    grouped kernel compiled for 6 waves per SIMD (VGPRs capped at 80); ``"grouped_h"``:
    the grouped kernel with each wave's (done, pos, slot) loaded once at entry;
    ``"mfma"``: single-pass transposed MFMA kernel (S^T = K·Q^T, O^T = V^T·P^T);
    ``"mfma_v1"``: S = Q·K^T with P through LDS; ``"valu"``: vector-ALU variant —
    kept for A/B measurement; ``"split2"``/``"split4"``/``"split8"``: key-split, N
    waves per (row, kv head) share the row's key tiles and merge their softmax
    states in LDS (the small-batch kernel: many short waves instead of few long
    ones).  MFMA kernels need ``Lmax``, padded prefix % 32 == 0."""
    B, nh, D = q.shape
    S, nkv, Lmax, _ = k_cache.shape
    P0pad = pk.shape[1]
    assert pos.numel() == B and slot.numel() == B and (done is None or done.numel() >= B)
    assert vt_cache.shape == vt_shape(S, nkv, D, Lmax) and pvt.shape == vt_shape(1, nkv, D, P0pad)[1:]
    lib = load_library()
    if impl == "cascade":
        if scratch is None:
            scratch = (torch.empty(B, nh, D, dtype=torch.float32, device=q.device),
                       torch.empty(B, nh, dtype=torch.float32, device=q.device))
        pre_o, pre_lse = scratch
        if (pre_o.dtype != torch.float32 or pre_lse.dtype != torch.float32 or pre_o.shape[0] < B
                or pre_o.shape[1:] != (nh, D) or pre_lse.shape[0] < B or pre_lse.shape[1:] != (nh,)):
            raise ValueError("attn_decode: bad cascade scratch")
        rc = lib.sg_attn_decode_cascade(_p(q), _p(pos), _p(slot), _p(done), _p(k_cache), _p(vt_cache), _p(pk),
                                        _p(pvt), P0, P0pad, _p(out), B, nh, nkv, D, Lmax, scale, _p(pre_o),
                                        _p(pre_lse), _stream())
        _check(rc, "attn_decode[cascade]")
        return out
    if impl.startswith("split"):
        nwv = int(impl[5:])
        if nwv not in (2, 4, 8):
            raise ValueError(f"attn_decode: {impl!r} (split2 / split4 / split8)")
        _check(lib.sg_attn_decode_split(_p(q), _p(pos), _p(slot), _p(done), _p(k_cache), _p(vt_cache), _p(pk),
                                        _p(pvt), P0, P0pad, _p(out), B, nh, nkv, D, Lmax, scale, nwv, _stream()),
               f"attn_decode[{impl}]")
        return out
    fn = {"mfma": lib.sg_attn_decode, "mfma_v1": lib.sg_attn_decode_v1, "valu": lib.sg_attn_decode_valu,
          "grouped": lib.sg_attn_decode_grouped, "grouped_pf": lib.sg_attn_decode_grouped_pf,
          "grouped6": lib.sg_attn_decode_grouped6, "grouped_h": lib.sg_attn_decode_grouped_h}[impl]
    _check(fn(_p(q), _p(pos), _p(slot), _p(done), _p(k_cache), _p(vt_cache), _p(pk), _p(pvt), P0, P0pad, _p(out), B,
              nh, nkv, D, Lmax, scale, _stream()), f"attn_decode[{impl}]")
    return out


def attn_spec(q: torch.Tensor, row_start: torch.Tensor, row_nd: torch.Tensor, x_pos: torch.Tensor,
              x_slot: torch.Tensor, x_done: torch.Tensor, k_cache: torch.Tensor, vt_cache: torch.Tensor,
              pk: torch.Tensor, pvt: torch.Tensor, P0: int, out: torch.Tensor, scale: float, max_q: int) -> torch.Tensor:
    """Decode attention of speculative pseudo-rows, one wave per (row, kv head).

    ``q`` / ``out`` = ``[T, nh, D]`` pseudo-rows as packed by :func:`spec_plan`: row
    ``r`` owns ``row_start[r] .. row_start[r] + row_nd[r]``, all on the row's KV slot,
    pseudo-row ``i`` attending to the prefix plus own keys ``[0, pos + i]``.  The row's
    key tiles are read once for all its pseudo-rows; per pseudo-row the result is
    bit-identical to ``attn_decode(impl="grouped")``.  Needs ``max_q * nh / nkv <= 32``
    (``max_q`` = 1 + the engine's spec_k; above 16 columns a wave runs two MFMA
    column blocks over the same key tiles)."""
    T, nh, D = q.shape
    S, nkv, Lmax, _ = k_cache.shape
    P0pad = pk.shape[1]
    B = row_start.numel()
    assert row_nd.numel() == B and x_pos.numel() >= T and x_slot.numel() >= T and x_done.numel() >= T
    assert out.shape[0] >= T and vt_cache.shape == vt_shape(S, nkv, D, Lmax)
    if not 1 <= max_q or max_q * (nh // nkv) > 32:
        raise ValueError(f"attn_spec: {max_q} pseudo-rows x {nh // nkv} heads do not fit one wave's 32 columns")
    _check(load_library().sg_attn_spec(_p(q), _p(row_start), _p(row_nd), _p(x_pos), _p(x_slot), _p(x_done),
                                       _p(k_cache), _p(vt_cache), _p(pk), _p(pvt), P0, P0pad, _p(out), B, nh, nkv, D,
                                       Lmax, scale, max_q, _stream()), "attn_spec")
    return out


def _copy_args(fsm, row_masks: Optional[torch.Tensor], rows: int, name: str):
    """(copy_kind, row_masks) pointers for a kernel that honours copy masks, or (None, None)."""
    if row_masks is None:
        return None, None
    if row_masks.dtype != torch.int32 or not row_masks.is_contiguous() or row_masks.dim() != 2 \
            or row_masks.shape[0] < rows or row_masks.shape[1] != fsm.vocab // 32 or fsm.copy_kind_t is None:
        raise ValueError(f"{name}: row_masks must be int32 [>= {rows}, {fsm.vocab // 32}] (ops.copy_masks)")
    return _p(fsm.copy_kind_t), _p(row_masks)


def fsm_sample(logits: torch.Tensor, fsm, state: torch.Tensor, tok_io: torch.Tensor, out_buf: torch.Tensor,
               out_len: torch.Tensor, done: torch.Tensor, pos: torch.Tensor, slot_id: torch.Tensor,
               temperature: float, seed: int, row_map: Optional[torch.Tensor] = None,
               row_masks: Optional[torch.Tensor] = None) -> None:
    """Masked argmax/Gumbel sampling + FSM transition for ``B = logits.shape[0]`` rows.

    Logits row ``i`` updates state row ``row_map[i]`` (or ``i``).  ``row_masks``
    (:func:`copy_masks`, one row per logits row): rows in copy states use their own mask."""
    B, V = logits.shape
    ldl = logits.stride(0)
    assert logits.dtype == torch.bfloat16 and logits.stride(1) == 1
    max_out = out_buf.shape[1]
    inv_t = 0.0 if temperature <= 0 else 1.0 / temperature
    ck, rm = _copy_args(fsm, row_masks, B, "fsm_sample")
    _check(load_library().sg_fsm_sample(
        _p(logits), ldl, _p(fsm.masks), _p(fsm.state_mask), _p(state), _p(fsm.next_sep_t), _p(fsm.next_tok_t),
        _p(fsm.enum_tok_t), _p(fsm.enum_next_t), fsm.E, fsm.sep_token, fsm.done_state, _p(tok_io), _p(out_buf),
        _p(out_len), _p(done), _p(pos), _p(slot_id), _p(row_map), max_out, V, B, inv_t, seed & 0xFFFFFFFF,
        ck, rm, _stream()),
        "fsm_sample")


def copy_masks(fsm, row_state: torch.Tensor, prev_tok: torch.Tensor, row_slot: torch.Tensor,
               body_buf: torch.Tensor, body_len: torch.Tensor, out: torch.Tensor, n: Optional[int] = None) -> torch.Tensor:
    """Per-row allowed-token masks of copy-constrained decoding (csrc/spec_kernels.hip
    ``copy_mask_kernel``): for each of ``n`` rows whose state is a copy state, ``out[r]``
    = the state's schema mask AND, at a value's first position, <sep> or any body token
    at a word boundary; after that, a token following ``prev_tok[r]`` in the body, and
    <sep> where such an occurrence is followed by a word boundary
    (:meth:`~smsgate_amd.serving.fsm.SchemaFSM.copy_mask_host` is the reference).  The
    body of row ``r`` is ``body_buf[row_slot[r], :body_len[row_slot[r]]]``.  Rows in
    other states are not written (the consumers only read copy rows)."""
    n = row_state.numel() if n is None else n
    if fsm.span:
        raise ValueError("copy_masks: the span format is decoded by sparse_argmax only")
    S1, LB = body_buf.shape
    for name, t in (("row_state", row_state), ("prev_tok", prev_tok), ("row_slot", row_slot)):
        _req(t, torch.int32, name)
        if t.numel() < n:
            raise ValueError(f"copy_masks: {name} has fewer than {n} rows")
    _req(body_buf, torch.int32, "body_buf")
    _req(body_len, torch.int32, "body_len")
    _req(out, torch.int32, "out")
    if out.dim() != 2 or out.shape[0] < n or out.shape[1] != fsm.vocab // 32 or body_len.numel() != S1:
        raise ValueError("copy_masks: out must be [>= n, vocab/32]; body_len must match body_buf")
    if fsm.copy_kind_t is None or fsm.tok_flags_t is None:
        raise ValueError("copy_masks: the FSM has no copy tables (to_device first)")
    _check(load_library().sg_copy_masks(_p(fsm.masks), _p(fsm.state_mask), fsm.sep_token, fsm.vocab,
                                        _p(fsm.copy_kind_t), _p(fsm.tok_flags_t), _p(row_state), _p(prev_tok),
                                        _p(row_slot),
                                        _p(body_buf), _p(body_len), LB, n, _p(out), _stream()), "copy_masks")
    return out


def ref_copy_masks(fsm, row_state, prev_tok, row_slot, body_buf, body_len) -> torch.Tensor:
    """fp32-free reference of :func:`copy_masks`: [n, vocab] bool (rows in non-copy
    states get their schema mask)."""
    import numpy as np

    st, pv, sl = (t.cpu().numpy() for t in (row_state, prev_tok, row_slot))
    bb, bl = body_buf.cpu().numpy(), body_len.cpu().numpy()
    rows = [fsm.copy_mask_host(int(st[r]), int(pv[r]), bb[sl[r], : bl[sl[r]]].tolist()) for r in range(len(st))]
    return torch.from_numpy(np.stack(rows)) if rows else torch.zeros(0, fsm.vocab, dtype=torch.bool)


def unpack_masks(words: torch.Tensor) -> torch.Tensor:
    """int32 [n, V/32] bit masks -> bool [n, V] (bit j of word w = token 32w + j)."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = (w.unsqueeze(-1) >> torch.arange(32, device=words.device)) & 1
    return bits.reshape(words.shape[0], -1).bool()


SPEC_MAX_K = 8


def _fsm_args(fsm):
    return (_p(fsm.masks), _p(fsm.state_mask), _p(fsm.next_sep_t), _p(fsm.next_tok_t), _p(fsm.enum_tok_t),
            _p(fsm.enum_next_t), fsm.E)


def spec_plan(fsm, state: torch.Tensor, x_state: torch.Tensor, K: int, T_cap: int, sep_token: int,
              scratch_slot: int, tok_buf: torch.Tensor, pos: torch.Tensor,
              slot: torch.Tensor, done: torch.Tensor, out_buf: torch.Tensor, out_len: torch.Tensor,
              body_buf: torch.Tensor, body_len: torch.Tensor, delim: torch.Tensor, draft_buf: torch.Tensor,
              x_tok: torch.Tensor, x_pos: torch.Tensor, x_slot: torch.Tensor, x_done: torch.Tensor,
              row_start: torch.Tensor, row_nd: torch.Tensor, meta: torch.Tensor, policy: int = 1) -> None:
    """Prompt-lookup drafts for ``B = tok_buf.numel()`` rows packed into ``T_cap``
    pseudo-rows (``csrc/spec_kernels.hip``); drafts follow the schema FSM from each
    row's ``state`` and ``x_state`` gets every pseudo-row's state.  All int32
    except ``delim`` (uint8 [V]).  ``policy`` 0: copy until the first <sep>; 1: also
    schema-forced tokens, implicit value ends, across <sep> and from field starts
    (spec_draft_kernel)."""
    B = tok_buf.numel()
    _req(state, torch.int32, "state")
    _req(x_state, torch.int32, "x_state")
    if state.numel() < B or x_state.numel() < T_cap:
        raise ValueError("spec_plan: state / x_state too small")
    S1, LB = body_buf.shape
    for name, t in (("tok_buf", tok_buf), ("pos", pos), ("slot", slot), ("done", done), ("out_len", out_len),
                    ("row_start", row_start), ("row_nd", row_nd)):
        _req(t, torch.int32, name)
        if t.numel() < B:
            raise ValueError(f"spec_plan: {name} has {t.numel()} < {B} rows")
    for name, t in (("x_tok", x_tok), ("x_pos", x_pos), ("x_slot", x_slot), ("x_done", x_done)):
        _req(t, torch.int32, name)
        if t.numel() < T_cap:
            raise ValueError(f"spec_plan: {name} smaller than T_cap")
    _req(out_buf, torch.int32, "out_buf")
    _req(body_buf, torch.int32, "body_buf")
    _req(body_len, torch.int32, "body_len")
    _req(delim, torch.uint8, "delim")
    _req(draft_buf, torch.int32, "draft_buf")
    _req(meta, torch.int32, "meta")
    if not (0 <= K <= SPEC_MAX_K) or T_cap < B or draft_buf.numel() < B * SPEC_MAX_K or body_len.numel() != S1:
        raise ValueError("spec_plan: bad K / T_cap / draft_buf / body_len")
    if not (0 <= scratch_slot < S1) or out_buf.shape[0] < B:
        raise ValueError("spec_plan: bad scratch slot / out_buf")
    _check(load_library().sg_spec_plan(
        *_fsm_args(fsm), fsm.done_state, fsm.vocab, _p(state), _p(x_state),
        B, K, T_cap, sep_token, scratch_slot, _p(tok_buf), _p(pos), _p(slot), _p(done), _p(out_buf), _p(out_len),
        out_buf.shape[1], _p(body_buf), _p(body_len), LB, _p(delim), _p(fsm.forced_t), int(policy), _p(draft_buf),
        _p(x_tok), _p(x_pos),
        _p(x_slot), _p(x_done), _p(row_start), _p(row_nd), _p(meta), _stream()), "spec_plan")


def spec_verify(logits: torch.Tensor, fsm, state: torch.Tensor, tok_buf: torch.Tensor, out_buf: torch.Tensor,
                out_len: torch.Tensor, done: torch.Tensor, pos: torch.Tensor, x_tok: torch.Tensor,
                row_start: torch.Tensor, row_nd: torch.Tensor, accepted: Optional[torch.Tensor] = None,
                row_masks: Optional[torch.Tensor] = None) -> None:
    """Greedy FSM-masked verification of the drafts of ``B = tok_buf.numel()`` rows
    (``logits`` [T_cap, V] over the pseudo-rows :func:`spec_plan` laid out).
    ``row_masks``: the pseudo-rows' copy masks (:func:`copy_masks`)."""
    B = tok_buf.numel()
    T, V = logits.shape
    if logits.dtype != torch.bfloat16 or logits.stride(1) != 1 or x_tok.numel() < T:
        raise ValueError("spec_verify: bad logits / x_tok")
    for name, t in (("state", state), ("out_len", out_len), ("done", done), ("pos", pos), ("row_start", row_start),
                    ("row_nd", row_nd)):
        if t.numel() < B or t.dtype != torch.int32:
            raise ValueError(f"spec_verify: bad {name}")
    if accepted is not None and (accepted.numel() < B or accepted.dtype != torch.int32):
        raise ValueError("spec_verify: bad accepted")
    ck, rm = _copy_args(fsm, row_masks, T, "spec_verify")
    _check(load_library().sg_spec_verify(
        _p(logits), logits.stride(0), _p(fsm.masks), _p(fsm.state_mask), _p(state), _p(fsm.next_sep_t),
        _p(fsm.next_tok_t), _p(fsm.enum_tok_t), _p(fsm.enum_next_t), fsm.E, fsm.sep_token, fsm.done_state,
        _p(tok_buf), _p(out_buf), _p(out_len), _p(done), _p(pos), _p(x_tok), _p(row_start), _p(row_nd),
        _p(accepted), out_buf.shape[1], V, B, ck, rm, _stream()), "spec_verify")


def gemm_argmax(a: torch.Tensor, w: torch.Tensor, row_state: torch.Tensor, fsm, best: torch.Tensor,
                norm_eps: Optional[float] = None, cfg: Optional[int] = None,
                ss_in: Optional[torch.Tensor] = None, row_masks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """lm_head GEMM with the schema-FSM masked arg-max fused in (EPI 4): for every
    row, ``best[row] = max(argmax_key(bf16 logit, token))`` over the tokens its FSM
    state allows — no logits are written.  ``w`` [V, K] (final norm folded in when
    ``norm_eps``); ``best`` uint64-as-int64 [>= M] is ZEROED here first.
    ``row_masks`` (:func:`copy_masks`): rows in copy states use their own mask row."""
    M, K = a.shape
    N = w.shape[0]
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or a.stride(1) != 1 or a.stride(0) % 8:
        raise ValueError("gemm_argmax: bf16 activations with 16-B aligned rows required")
    if not w.is_contiguous() or w.shape[1] != K or K % 64 or N % 128 or N != fsm.vocab:
        raise ValueError(f"gemm_argmax: bad weight {tuple(w.shape)} for vocab {fsm.vocab}")
    _req(row_state, torch.int32, "row_state")
    if row_state.numel() < M or best.dtype != torch.int64 or best.numel() < M or not best.is_contiguous():
        raise ValueError("gemm_argmax: row_state / best too small or best not int64")
    best[:M].zero_()
    if M == 0:
        return best
    if cfg is None:
        cfg = 0 if -(-M // 128) * (N // 128) >= 480 else (3 if M > 1024 else 17)
    if ss_in is not None and norm_eps is None:
        raise ValueError("gemm_argmax: ss_in needs norm_eps")
    ld = _ss_check(ss_in, M, "gemm_argmax ss_in")
    norm = 0 if norm_eps is None else (2 if ss_in is not None else 1)
    ck, rm = _copy_args(fsm, row_masks, M, "gemm_argmax")
    _check(load_library().sg_gemm_argmax(_p(a), a.stride(0), _p(w), M, N, K, float(norm_eps or 0.0),
                                         norm, cfg, _p(row_state), _p(fsm.state_mask),
                                         _p(fsm.masks), _p(best), _p(ss_in), ld, ck, rm, _stream()), "gemm_argmax")
    return best


def embed_rows(ids: torch.Tensor, table: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``table[ids]`` for int32 ``ids`` (one kernel; ``F.embedding`` needs int64 ids, i.e.
    a cast and a gather per call); ids outside the table give zero rows."""
    _req(ids, torch.int32, "ids")
    V, H = table.shape
    if table.dtype != torch.bfloat16 or not table.is_contiguous() or H % 8:
        raise ValueError("embed_rows: contiguous bf16 table with H % 8 == 0 required")
    T = ids.numel()
    if out is None:
        out = table.new_empty((T, H))
    if out.shape != (T, H) or not out.is_contiguous() or out.dtype != torch.bfloat16:
        raise ValueError("embed_rows: bad output")
    _check(load_library().sg_embed_rows(_p(ids), _p(table), _p(out), T, H, V, _stream()), "embed_rows")
    return out


def embed_rows_add(ids: torch.Tensor, pos: torch.Tensor, table: torch.Tensor, base: int) -> torch.Tensor:
    """``table[ids] + table[base + pos]`` (int32 ids / positions, bf16 rows; the sum
    rounded like torch's bf16 add) -- the span format's prompt rows, one kernel."""
    _req(ids, torch.int32, "ids")
    _req(pos, torch.int32, "pos")
    V, H = table.shape
    if table.dtype != torch.bfloat16 or not table.is_contiguous() or H % 8 or pos.numel() != ids.numel():
        raise ValueError("embed_rows_add: contiguous bf16 table with H % 8 == 0 and one position per id required")
    T = ids.numel()
    out = table.new_empty((T, H))
    _check(load_library().sg_embed_rows_add(_p(ids), _p(pos), _p(table), _p(out), T, H, V, int(base), _stream()),
           "embed_rows_add")
    return out


QA_MAX_NF, QA_MAX_NQ, QA_MAX_POS, QA_NCLS, QA_MAX_CLS_TOK = 8, 24, 160, 4, 8


class QAParams(ctypes.Structure):
    """``QAParams`` of csrc/qa_kernels.hip (plain ints, same order)."""
    _fields_ = [("nf", _c_int), ("nq", _c_int), ("n_pos", _c_int),
                ("start_row", _c_int * QA_MAX_NF), ("end_row", _c_int * QA_MAX_NF),
                ("cls_bits", _c_int * QA_MAX_NF), ("cap", _c_int * QA_MAX_NF),
                ("off_end", _c_int), ("off_null", _c_int), ("off_cls", _c_int),
                ("cls_tok", (_c_int * QA_MAX_CLS_TOK) * QA_NCLS), ("cls_len", _c_int * QA_NCLS),
                ("reject_mask", _c_int), ("sep", _c_int), ("max_out", _c_int),
                ("s_need", _c_int * QA_MAX_NF), ("e_need", _c_int * QA_MAX_NF), ("absorb", _c_int * QA_MAX_NF),
                ("min_conf", _c_float), ("abstain_cls", _c_int)]


def qa_params(lay, tokenizer, min_conf: float = 0.0) -> QAParams:
    """Kernel parameters of a qa layout (serving/qa.py): query rows, field classes and
    caps, the W row offsets (W = rows ptr0 .. cls0 + 3 of the final-norm-folded
    embedding), the class tokens of the copy-format answer, and the abstention
    threshold (``min_conf``: a transaction answer less confident than this becomes the
    ``unknown`` class; 0 = never)."""
    from ..parse.schema import TXN_TYPES
    from ..serving.qa import ABSTAIN_TXN, REJECT_TXN, qa_rows

    p = QAParams()
    nf = lay.n_copy
    if nf > QA_MAX_NF or lay.n_queries > QA_MAX_NQ or lay.n_pos > QA_MAX_POS:
        raise ValueError("qa_params: layout exceeds the kernel's limits")
    p.nf, p.nq, p.n_pos = nf, lay.n_queries, lay.n_pos
    srows, erows = qa_rows(lay)
    for f in range(nf):
        p.start_row[f], p.end_row[f] = srows[f], erows[f]
        p.cls_bits[f], p.cap[f], p.s_need[f], p.e_need[f] = lay.rules()[f]
        p.absorb[f] = int(lay.absorb_time()[f])
    p.off_end, p.off_null, p.off_cls = lay.pe0 - lay.ptr0, lay.null_id - lay.ptr0, lay.cls0 - lay.ptr0
    for c, name in enumerate(TXN_TYPES):
        toks = tokenizer.encode(name)
        if not 0 < len(toks) <= QA_MAX_CLS_TOK:
            raise ValueError(f"qa_params: class {name!r} encodes to {len(toks)} tokens")
        for k, t in enumerate(toks):
            p.cls_tok[c][k] = t
        p.cls_len[c] = len(toks)
        if name in REJECT_TXN:
            p.reject_mask |= 1 << c
    p.sep, p.max_out = tokenizer.sep, lay.max_answer_tokens()
    p.min_conf, p.abstain_cls = float(min_conf), TXN_TYPES.index(ABSTAIN_TXN)
    if load_library().sg_qa_params_size() != ctypes.sizeof(QAParams):
        raise RuntimeError("QAParams layout differs from csrc/qa_kernels.hip")
    return p


def qa_decode(h: torch.Tensor, W: torch.Tensor, eps: float, cu: torch.Tensor, ids: torch.Tensor,
              flags: torch.Tensor, params: QAParams, out_buf: torch.Tensor, out_len: torch.Tensor,
              dbg_scores: Optional[torch.Tensor] = None, dbg_spans: Optional[torch.Tensor] = None,
              compact: bool = False, out_conf: Optional[torch.Tensor] = None) -> None:
    """The qa format's head (``qa_decode_kernel``): for every sequence ``m`` of a packed
    prefill batch (rows ``cu[m]:cu[m+1]``, the last ``params.nq`` of them its query
    rows; ``compact``: ``h`` holds only the query rows, ``m * nq ..``), scores of the query rows against W (RMSNorm from the un-normed rows ``h``,
    weight folded into W), the class and every field's joint constrained span decode,
    and the answer in the copy format into ``out_buf[m]`` / ``out_len[m]``.
    ``dbg_scores`` [M, 4 + nf (2 n_pos + 1)] fp32 / ``dbg_spans`` [M, 1 + 2 nf] int32:
    the raw scores and the decoded (class, start, end ...) for tests.  ``out_conf`` [M]
    fp32: each answer's confidence (the least probable of its decisions; before the
    ``params.min_conf`` abstention)."""
    M = cu.numel() - 1
    T, H = h.shape[0], h.shape[1]
    if h.dtype != torch.bfloat16 or h.stride(1) != 1 or h.stride(0) % 8 or not h.is_cuda:
        raise ValueError("qa_decode: bf16 rows with 16-B aligned strides required")
    R = params.off_cls + QA_NCLS
    if W.dtype != torch.bfloat16 or not W.is_contiguous() or W.shape[1] != H or W.shape[0] < R:
        raise ValueError(f"qa_decode: W must be bf16 [>= {R}, {H}]")
    for t, name in ((cu, "cu"), (ids, "ids"), (out_len, "out_len")):
        _req(t, torch.int32, name)
    if compact and T < M * params.nq:
        raise ValueError("qa_decode: compact h needs nq rows per sequence")
    if out_len.numel() < M or out_buf.dtype != torch.int32 or not out_buf.is_contiguous() or (
            not compact and ids.numel() < T):
        raise ValueError("qa_decode: ids / out_len / out_buf too small")
    if out_buf.dim() != 2 or out_buf.shape[0] < M or out_buf.shape[1] != params.max_out:
        raise ValueError(f"qa_decode: out_buf must be int32 [>= {M}, {params.max_out}]")
    if flags.dtype not in (torch.int32, torch.uint32) or not flags.is_contiguous():
        raise ValueError("qa_decode: flags must be a contiguous 32-bit table (serving/qa.py qa_token_flags)")
    per = QA_NCLS + params.nf * (2 * params.n_pos + 1)
    if dbg_scores is not None and (dbg_scores.dtype != torch.float32 or dbg_scores.numel() < M * per):
        raise ValueError(f"qa_decode: dbg_scores must be fp32 [{M}, {per}]")
    if dbg_spans is not None and (dbg_spans.dtype != torch.int32 or dbg_spans.numel() < M * (1 + 2 * params.nf)):
        raise ValueError("qa_decode: dbg_spans too small")
    if out_conf is not None and (out_conf.dtype != torch.float32 or out_conf.numel() < M or not out_conf.is_cuda):
        raise ValueError("qa_decode: out_conf must be fp32 [>= M] on the GPU")
    if M == 0:
        return
    _check(load_library().sg_qa_decode(ctypes.byref(params), _p(h), h.stride(0), _p(W), H, float(eps), _p(cu),
                                       _p(ids), _p(flags), flags.numel(), _p(out_buf), _p(out_len), _p(dbg_scores),
                                       _p(dbg_spans), _p(out_conf), M, int(bool(compact)), _stream()), "qa_decode")


def embed_rows_add_ids(ids: torch.Tensor, add: torch.Tensor, table: torch.Tensor,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``table[ids] + table[add]`` (no second row where ``add < 0``), bf16 rounded like
    torch's add -- the qa format's prompt rows (pointer rows on message tokens only)."""
    _req(ids, torch.int32, "ids")
    _req(add, torch.int32, "add")
    V, H = table.shape
    if table.dtype != torch.bfloat16 or not table.is_contiguous() or H % 8 or add.numel() != ids.numel():
        raise ValueError("embed_rows_add_ids: contiguous bf16 table with H % 8 == 0 and one add id per id")
    T = ids.numel()
    if out is None:
        out = table.new_empty((T, H))
    _check(load_library().sg_embed_rows_add_ids(_p(ids), _p(add), _p(table), _p(out), T, H, V, _stream()),
           "embed_rows_add_ids")
    return out


def sparse_argmax(h: torch.Tensor, w: torch.Tensor, row_state: torch.Tensor, fsm, best: torch.Tensor,
                  prev_tok: torch.Tensor, row_slot: torch.Tensor, body_buf: torch.Tensor, body_len: torch.Tensor,
                  eps: float) -> torch.Tensor:
    """Candidate-sparse lm_head + masked arg-max (``sparse_argmax_kernel``): ``best[r]``
    = :func:`gemm_argmax`'s key over the tokens row ``r`` may emit — the schema mask of
    its state, AND in a copy state the tokens its SMS body allows after ``prev_tok[r]``
    (:func:`copy_masks`' rules) — computed from those candidates' lm_head rows only.
    ``h`` [n, H] un-normed rows, ``w`` [V, H] with the final RMSNorm weight folded in
    (:func:`fold_norm`); the row scale is computed from ``h``."""
    n, H = h.shape
    if h.dtype != torch.bfloat16 or h.stride(1) != 1 or h.stride(0) % 8 or not w.is_contiguous():
        raise ValueError("sparse_argmax: bf16 rows with 16-B aligned strides and a contiguous weight required")
    if w.shape != (fsm.vocab, H) or H % 64 or H > 1024:
        raise ValueError(f"sparse_argmax: weight {tuple(w.shape)} vs vocab {fsm.vocab}, hidden {H}")
    for t, name in ((row_state, "row_state"), (prev_tok, "prev_tok"), (row_slot, "row_slot")):
        _req(t, torch.int32, name)
        if t.numel() < n:
            raise ValueError(f"sparse_argmax: {name} shorter than the rows")
    if best.dtype != torch.int64 or best.numel() < n or not best.is_contiguous():
        raise ValueError("sparse_argmax: best must be int64 [>= n]")
    if n == 0:
        return best
    _req(body_buf, torch.int32, "body_buf")
    ck = _p(fsm.copy_kind_t) if fsm.has_copy else None
    _check(load_library().sg_sparse_argmax(_p(fsm.masks), _p(fsm.state_mask), fsm.sep_token, fsm.vocab, ck,
                                           _p(fsm.tok_flags_t), _p(h), h.stride(0), _p(w), H, float(eps),
                                           _p(row_state), _p(prev_tok), _p(row_slot), _p(body_buf),
                                           _p(body_len), body_buf.shape[1], n, fsm.ptr0 if fsm.span else -1,
                                           fsm.n_pos if fsm.span else 0, _p(best), _stream()),
           "sparse_argmax")
    return best


def sparse_argmax_ok(fsm) -> bool:
    """The sparse arg-max needs every NON-copy state to allow at most 256 tokens (its
    candidate list; copy states allow at most the body's tokens + <sep>, < 256)."""
    ck = fsm.copy_kind if fsm.copy_kind is not None else np.zeros(fsm.num_states, dtype=np.int32)
    return int(fsm.allowed[ck == 0].sum(1).max(initial=0)) <= 256


def fsm_commit(best: torch.Tensor, fsm, state: torch.Tensor, tok_io: torch.Tensor, out_buf: torch.Tensor,
               out_len: torch.Tensor, done: torch.Tensor, pos: torch.Tensor, B: int,
               row_map: Optional[torch.Tensor] = None) -> None:
    """Greedy FSM step from :func:`gemm_argmax` keys (row ``i`` -> state row ``row_map[i]``)."""
    if best.dtype != torch.int64 or best.numel() < B or (row_map is not None and row_map.numel() < B):
        raise ValueError("fsm_commit: bad best / row_map")
    if row_map is None and state.numel() < B:
        raise ValueError("fsm_commit: state smaller than B")
    _check(load_library().sg_fsm_commit(
        _p(best), _p(row_map), *_fsm_args(fsm), fsm.sep_token, fsm.done_state, fsm.vocab, _p(state), _p(tok_io),
        _p(out_buf), _p(out_len), _p(done), _p(pos), out_buf.shape[1], B, _stream()), "fsm_commit")


def span_commit(best: torch.Tensor, fsm, state: torch.Tensor, tok_io: torch.Tensor, out_buf: torch.Tensor,
                out_len: torch.Tensor, done: torch.Tensor, pos: torch.Tensor, row_slot: torch.Tensor,
                body_buf: torch.Tensor, body_len: torch.Tensor, B: int, row_map: Optional[torch.Tensor] = None) -> None:
    """:func:`fsm_commit` of the span-pointer format (``span_commit_kernel``): the FSM
    step from the arg-max keys, and the answer written in COPY format -- an end
    pointer appends its span's body tokens (``body_buf[row_slot[i]]``) and <sep>.
    :meth:`~smsgate_amd.serving.fsm.SchemaFSM.expand_span_answer` is the reference."""
    if not fsm.span:
        raise ValueError("span_commit: not a span-format FSM")
    if best.dtype != torch.int64 or best.numel() < B or (row_map is not None and row_map.numel() < B):
        raise ValueError("span_commit: bad best / row_map")
    if row_map is None and state.numel() < B:
        raise ValueError("span_commit: state smaller than B")
    _req(row_slot, torch.int32, "row_slot")
    _req(body_buf, torch.int32, "body_buf")
    _req(body_len, torch.int32, "body_len")
    if row_slot.numel() < B or body_len.numel() != body_buf.shape[0]:
        raise ValueError("span_commit: bad row_slot / body_len")
    _check(load_library().sg_span_commit(
        _p(best), _p(row_map), *_fsm_args(fsm), fsm.sep_token, fsm.done_state, fsm.vocab, _p(fsm.copy_kind_t),
        _p(row_slot), _p(body_buf), _p(body_len), body_buf.shape[1], fsm.ptr0, _p(state), _p(tok_io), _p(out_buf),
        _p(out_len), _p(done), _p(pos), out_buf.shape[1], B, _stream()), "span_commit")


def spec_verify_keys(best: torch.Tensor, fsm, state: torch.Tensor, tok_buf: torch.Tensor, out_buf: torch.Tensor,
                     out_len: torch.Tensor, done: torch.Tensor, pos: torch.Tensor, x_tok: torch.Tensor,
                     row_start: torch.Tensor, row_nd: torch.Tensor, accepted: Optional[torch.Tensor] = None,
                     counts: Optional[torch.Tensor] = None) -> None:
    """Greedy verification of the drafts from :func:`gemm_argmax` keys (one thread per row).
    ``counts`` (int64 [2], optional): += (tokens emitted, rows that emitted) of this step."""
    if counts is not None and (counts.dtype != torch.int64 or counts.numel() < 2 or not counts.is_contiguous()):
        raise ValueError("spec_verify_keys: counts must be a contiguous int64 [2]")
    B = tok_buf.numel()
    if best.dtype != torch.int64 or best.numel() < x_tok.numel():
        raise ValueError("spec_verify_keys: best must cover every pseudo-row")
    for name, t in (("state", state), ("out_len", out_len), ("done", done), ("pos", pos), ("row_start", row_start),
                    ("row_nd", row_nd)):
        if t.numel() < B or t.dtype != torch.int32:
            raise ValueError(f"spec_verify_keys: bad {name}")
    _check(load_library().sg_spec_verify_keys(
        _p(best), *_fsm_args(fsm), fsm.sep_token, fsm.done_state, fsm.vocab, _p(state), _p(tok_buf), _p(out_buf),
        _p(out_len), _p(done), _p(pos), _p(x_tok), _p(row_start), _p(row_nd), _p(accepted), out_buf.shape[1], B,
        _p(counts), _stream()), "spec_verify_keys")


def kv_copy_prefix(k_cache: torch.Tensor, vt_cache: torch.Tensor, items: torch.Tensor) -> None:
    """Copy own offsets ``0..k-1`` of each item's template slot into its message slot,
    every layer (keys row-wise, Vᵀ as whole 8-key blocks).  ``k_cache`` [L, S, nkv,
    Lmax, 64], ``vt_cache`` its blocked Vᵀ twin, ``items`` int32 [3, n] = (template
    slot, message slot, k)."""
    L, S, nkv, Lmax, D = k_cache.shape
    assert vt_cache.shape == (L, *vt_shape(S, nkv, D, Lmax)) and k_cache.is_contiguous() and vt_cache.is_contiguous()
    _req(items, torch.int32, "items")
    assert items.dim() == 2 and items.shape[0] == 3 and items.is_contiguous()
    n = items.shape[1]
    _check(load_library().sg_kv_copy_prefix(_p(k_cache), _p(vt_cache), _p(items), n, L, S, nkv, D, Lmax,
                                            _stream()), "kv_copy_prefix")


def vt_shape(S: int, nkv: int, D: int, L: int):
    """Blocked V^T cache layout ``[S][nkv][L/8][D][8]`` (8 keys of one dim = 16 bytes)."""
    assert L % 8 == 0
    return (S, nkv, L // 8, D, 8)


def vt_to_rows(vt: torch.Tensor) -> torch.Tensor:
    """Blocked ``[..., L/8, D, 8]`` → plain rows ``[..., L, D]`` (tests/debugging)."""
    *lead, nb, D, eight = vt.shape
    return vt.transpose(-1, -2).reshape(*lead, nb * eight, D)


def rows_to_vt(v: torch.Tensor) -> torch.Tensor:
    """Plain rows ``[..., L, D]`` → blocked ``[..., L/8, D, 8]``."""
    *lead, L, D = v.shape
    return v.reshape(*lead, L // 8, 8, D).transpose(-1, -2).contiguous()


# ------------------------------------------------------------------ references
def ref_rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def ref_silu_mul(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return torch.nn.functional.silu(g) * u


def ref_rope(x: torch.Tensor, positions: torch.Tensor, theta: float) -> torch.Tensor:
    """rotate-half RoPE in fp32; ``x``: [T, H, D], ``positions``: [T]."""
    D = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64, device=x.device) / D))
    ang = positions.double()[:, None] * inv[None, :]
    cos, sin = ang.cos().float()[:, None, :], ang.sin().float()[:, None, :]
    x1, x2 = x.float()[..., : D // 2], x.float()[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def ref_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, mask: torch.Tensor, scale: float) -> torch.Tensor:
    """fp32 attention. q [nq, D], k/v [nk, D], mask [nq, nk] bool (True = attend)."""
    s = (q.float() @ k.float().t()) * scale
    s = s.masked_fill(~mask, float("-inf"))
    return torch.softmax(s, dim=-1) @ v.float()


def ref_gemm(a: torch.Tensor, w: torch.Tensor, *, epi: str = "store", norm_eps: Optional[float] = None,
             norm_w: Optional[torch.Tensor] = None, resid: Optional[torch.Tensor] = None,
             gate_up_plain: bool = True) -> torch.Tensor:
    """fp32 reference of :func:`gemm` on UN-folded, UN-interleaved weights:
    ``x = rmsnorm(a)·norm_w`` (if ``norm_eps``), ``y = x @ w.T``, then the epilogue."""
    x = a.float()
    if norm_eps is not None:
        x = ref_rmsnorm(x, norm_w if norm_w is not None else torch.ones(x.shape[1], device=x.device), norm_eps)
    y = x @ w.float().t()
    if epi == "swiglu":
        return ref_silu_mul(y)
    if epi == "resid":
        return resid.float() + y
    return y

