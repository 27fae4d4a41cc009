"""Build the native (host C++) components in-tree.

``python -m smsgate_amd.native.build`` (also run by ``__graft_entry__.build()``)
compiles ``csrc/busd.cpp`` into ``_bin/smsgate-busd``, the native bus broker
(see :mod:`smsgate_amd.native`).  Plain ``g++ -O2 -std=c++17``: no Python or
torch headers, no third-party libraries.  Skipped when the binary is newer than
every source.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path
from typing import List

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BINDIR = HERE / "_bin"
LIBDIR = HERE / "_lib"  # in-tree CPython extensions (git-ignored, travel with the tree)
BUSD = BINDIR / "smsgate-busd"
# host sanitizer build (ASan + UBSan): the broker's race/memory check, run by
# tests/test_native_bus.py::test_sanitizer_build_clean (GPU sanitizers are not used)
BUSD_SAN = BINDIR / "smsgate-busd-san"
# native load generator (broker capacity tests, scripts/bus_bench.py --native-load)
BUSLOAD = BINDIR / "smsgate-busload"


def cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++"), shutil.which("clang++")):
        if cand:
            return cand
    raise RuntimeError("no C++ compiler found")


# CPython extensions (one .cpp each), not part of the broker binary
EXTENSIONS = ("tokfast.cpp", "parsefast.cpp")


def sources() -> List[Path]:
    return sorted(p for p in CSRC.glob("*.cpp") if p.name not in EXTENSIONS) + sorted(CSRC.glob("*.hpp"))


def needs_build(target: Path = BUSD) -> bool:
    if not target.exists():
        return True
    mt = target.stat().st_mtime
    return any(s.stat().st_mtime > mt for s in sources() + [Path(__file__)])


def build_tokfast(force: bool = False, verbose: bool = False) -> Path:
    """``_lib/_tokfast*.so``: the CPython extension of ``csrc/tokfast.cpp`` (native
    BPE encoder / answer decoder of the parser processes, models/fasttok.py)."""
    return build_extension("tokfast", force, verbose)


def build_parsefast(force: bool = False, verbose: bool = False) -> Path:
    """``_lib/_parsefast*.so``: ``csrc/parsefast.cpp``, the parser processes' native
    per-message path (parse/fastpath.py)."""
    return build_extension("parsefast", force, verbose)


# libraries an extension links (the system OpenSSL the interpreter's hashlib uses)
LINK = {"parsefast": ["-lcrypto"]}


def build_extension(name: str, force: bool = False, verbose: bool = False) -> Path:
    import sysconfig

    LIBDIR.mkdir(parents=True, exist_ok=True)
    target = LIBDIR / ("_" + name + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    src = CSRC / f"{name}.cpp"
    deps = [src, Path(__file__)] + sorted(CSRC.glob("*.hpp"))
    if not force and target.exists() and target.stat().st_mtime > max(d.stat().st_mtime for d in deps):
        return target
    tmp = target.with_suffix(".tmp")
    cmd = [cxx(), "-O3", "-std=c++17", "-Wall", "-Wno-unused-function", "-shared", "-fPIC", "-fvisibility=hidden",
           f"-I{sysconfig.get_paths()['include']}", str(src), "-o", str(tmp)] + LINK.get(name, [])
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


def build(force: bool = False, verbose: bool = False, extra: List[str] = (), sanitize: bool = False) -> Path:
    if not sanitize:
        build_tokfast(force=force, verbose=verbose)
        build_parsefast(force=force, verbose=verbose)
    target = BUSD_SAN if sanitize else BUSD
    if not force and not needs_build(target):
        return target
    BINDIR.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".tmp")
    opt = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"] \
        if sanitize else ["-O2"]
    cmd = [cxx(), *opt, "-std=c++17", "-Wall", "-Wno-unused-function", "-pthread", *extra,
           str(CSRC / "busd.cpp"), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    if not sanitize:
        build_load(force=force, verbose=verbose)
    return target


def build_load(force: bool = False, verbose: bool = False) -> Path:
    """The native load generator (threads; one connection per producer / consumer)."""
    if not force and not needs_build(BUSLOAD):
        return BUSLOAD
    tmp = BUSLOAD.with_suffix(".tmp")
    cmd = [cxx(), "-O2", "-std=c++17", "-Wall", "-Wno-unused-function", "-pthread", str(CSRC / "busload.cpp"),
           "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, BUSLOAD)
    return BUSLOAD


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--sanitize" in sys.argv:
        print(build(force="--force" in sys.argv, verbose=True, sanitize=True))
