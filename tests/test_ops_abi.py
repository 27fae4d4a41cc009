"""CPU check: every ctypes declaration matches its extern "C" signature in the .hip
sources (a wrong argtypes list would corrupt a launch on the GPU box)."""
import re
from pathlib import Path

import pytest

from smsgate_amd import ops

CSRC = Path(ops.__file__).parent / "csrc"


def _c_signatures():
    sigs = {}
    for f in CSRC.glob("*.hip"):
        text = f.read_text()
        block = text[text.index('extern "C" {'):]
        for m in re.finditer(r"\b(?:int|void)\s+(sg_\w+)\s*\(([^)]*)\)\s*\{", block):
            args = [a.strip() for a in m.group(2).split(",") if a.strip()]
            sigs[m.group(1)] = args
    return sigs


class _FakeFn:
    argtypes = None
    restype = None


class _FakeLib:
    def __getattr__(self, name):
        fn = _FakeFn()
        object.__setattr__(self, name, fn)
        return fn


def test_argtypes_match_c_signatures():
    sigs = _c_signatures()
    lib = _FakeLib()
    ops._declare(lib)
    declared = {k: v for k, v in vars(lib).items() if isinstance(v, _FakeFn) and v.argtypes is not None}
    assert declared, "no declarations captured"
    for name, fn in declared.items():
        assert name in sigs, name
        c_args = sigs[name]
        assert len(fn.argtypes) == len(c_args), (name, len(fn.argtypes), c_args)
        for t, a in zip(fn.argtypes, c_args):
            if "*" in a or "hipStream_t" in a:
                assert t.__name__ in ("c_void_p",), (name, a, t)
            elif a.startswith("float"):
                assert t.__name__ == "c_float", (name, a, t)
            elif a.startswith("int") or a.startswith("unsigned"):
                assert t.__name__ in ("c_int", "c_uint"), (name, a, t)


@pytest.mark.parametrize("fn", ["sg_rmsnorm_residual", "sg_attn_prefill", "sg_attn_decode", "sg_fsm_sample", "sg_gemm"])
def test_expected_entry_points_exist(fn):
    assert fn in _c_signatures()


def test_row_partials_image_and_checks():
    """x² partials image: [SS_PARTS, M rounded up to 16-B row groups], validated before
    any launch (CPU tensors and wrong shapes are refused)."""
    import torch

    ss = ops.ss_buffer(10, "cpu")
    assert ss.shape == (ops.SS_PARTS, 12) and ss.dtype == torch.float32 and not ss.any()
    with pytest.raises(ValueError):
        ops._ss_check(ss, 10, "t")  # not on the GPU
    with pytest.raises(ValueError):
        ops._ss_check(torch.zeros(ops.SS_PARTS - 1, 16), 4, "t")
    assert ops._ss_check(None, 10, "t") == 0


def test_measured_tile_exceptions():
    """gate/up uses the staggered 256x256 kernels where measured faster (persistent
    form from 4096 rows), the 8-wave 128x128 tile just below."""
    if not ops.GEMM_MEASURED:
        pytest.skip("SMSGATE_GEMM_MEASURED=0")
    assert ops.gemm_cfg(9216, 3072, epi="swiglu", K=576) == 20
    assert ops.gemm_cfg(16384, 3072, epi="swiglu", K=576) == 20
    assert ops.gemm_cfg(2304, 3072, epi="swiglu", K=576) == 13
    assert ops.gemm_cfg(4608, 3072, epi="swiglu", K=576) == 19
    # o-proj and down-proj tile N in multiples of 96 columns at every row count: both then
    # write the producer-norm partials as the same six 96-column parts, whatever the tile
    for M in list(range(1, 40000, 97)) + [65536, 110592, 221184]:
        bn = {ops.GEMM_TILES[ops.gemm_cfg(M, 576, epi="resid", K=k)][1] for k in (576, 1536)}
        assert all(b % 96 == 0 for b in bn), (M, bn)
    assert ops.gemm_cfg(9216, 576, epi="resid", K=1536) == 21
    # the qa engine's batches: 128x192 (profiles/r05_gemm_tune_qa.json)
    assert ops.gemm_cfg(110592, 576, epi="resid", K=1536) == ops.gemm_cfg(110592, 576, epi="resid", K=576) == 28
    assert ops.GEMM_TILES[20] == (256, 256) and 20 in ops.GEMM_SWIGLU_ONLY
    assert all(576 % ops.GEMM_TILES[c][1] == 0 for c in ops.GEMM_NO_SWIGLU)  # the N = 576 residual GEMMs


def test_qkv_tile_rule():
    """The 3-head (192-wide) QKV tile only where both head counts divide by 3; 32-row
    tiles for small batches, 128x64 for prefill-sized ones."""
    from smsgate_amd import ops

    assert ops.qkv_cfg(9216, 9, 3) == 28
    assert ops.qkv_cfg(9216, 4, 2) == 3 and ops.qkv_cfg(9216, 9, 2) == 3
    assert ops.qkv_cfg(1000) == 17 and ops.qkv_cfg(4608) == 3 and ops.qkv_cfg(15104) == 1
    assert ops.qkv_cfg(110592) == 28 and ops.qkv_cfg(110592, 4, 2) == 1
    bm, bn = ops.GEMM_TILES[28]
    assert (bm, bn) == (128, 192) and 28 in ops.GEMM_NO_SWIGLU
