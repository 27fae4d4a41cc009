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
