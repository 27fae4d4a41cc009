"""Build the in-tree HIP kernel library for gfx950 with an explicit hipcc line.

``python -m smsgate_amd.ops.build`` (also run by ``__graft_entry__.build()``)
compiles every ``csrc/*.hip`` into ``_lib/libsmsgate_kernels.so``.  The
library exposes a plain C ABI and is loaded with ``ctypes`` — no torch C++
headers (fast builds, no ABI coupling, no hipify step) — and every launch
takes the caller's ``hipStream_t`` so it can be captured into a hipGraph.
The build is skipped when the .so is newer than all sources.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path
from typing import List, Optional

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIBDIR = HERE / "_lib"
LIB = LIBDIR / "libsmsgate_kernels.so"
ARCH = os.environ.get("SMSGATE_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm not installed?)")


def sources() -> List[Path]:
    return sorted(CSRC.glob("*.hip"))


def needs_build(lib: Path = LIB) -> bool:
    if not lib.exists():
        return True
    mt = lib.stat().st_mtime
    return any(s.stat().st_mtime > mt for s in sources() + [Path(__file__)])


def build(force: bool = False, verbose: bool = False, extra: Optional[List[str]] = None) -> Path:
    if not force and not needs_build():
        return LIB
    LIBDIR.mkdir(parents=True, exist_ok=True)
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [
        hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-munsafe-fp-atomics",
        # MFMA accumulators in VGPRs: the default AGPR form made the GEMM K-loop
        # shuffle its accumulators (68 v_accvgpr_* per 32 MFMAs) and cost the
        # attention kernels one wave of occupancy (scripts/kernel_resources.py)
        "-mllvm",
        "-amdgpu-mfma-vgpr-form=1",
        *(extra or []),
        *[str(s) for s in sources()],
        "-o",
        str(tmp),
    ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
