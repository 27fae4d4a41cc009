"""Native encoder / decoder of the extractor tokenizer (``native/csrc/tokfast.cpp``).

:class:`FastTokenizer` wraps the C++ module built from the SAME tokenizer file the
library loads (vocabulary, merge ranks, special tokens): it produces the engine's
wire format (uint16 lengths + int32 ids, serving/protocol.py) for a whole batch in
one call and decodes answer batches straight from the response buffer.
``tests/test_fasttok.py`` pins id-for-id equality with the ``tokenizers``
library on every template family and on random Unicode.

The pre-tokenizer's character classes come from :mod:`unicodedata` (letters
``L*``, numbers ``N*``, digits ``Nd`` -- the library's ``\\d`` is Unicode) plus
the whitespace set the library's ``\\s`` matches, probed against the library
itself at load (:func:`_whitespace`).  :func:`load_fast_tokenizer` returns None
when the extension is not built; callers then use the library path.
"""
from __future__ import annotations

import functools
import json
import os
import sys
import unicodedata
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

__all__ = ["FastTokenizer", "load_fast_tokenizer", "native_available"]

_HERE = Path(__file__).resolve().parent.parent / "native" / "_lib"
_L, _N, _D, _S = 1, 2, 4, 8


def _import_ext():
    p = str(_HERE)
    if p not in sys.path:
        sys.path.insert(0, p)
    try:
        import _tokfast  # type: ignore

        return _tokfast
    except ImportError:
        return None


def native_available() -> bool:
    return _import_ext() is not None


def _whitespace(pretok) -> List[int]:
    """Code points the library's ``\\s`` matches: ``"a" + c + c + "b"`` splits into
    four one-character pieces exactly when ``c`` is whitespace to the regex."""
    cands = {c for c in range(0x3000 + 1) if chr(c).isspace() or unicodedata.category(chr(c)) in ("Zs", "Zl", "Zp")}
    cands |= {0x180E, 0x200B, 0x2060, 0xFEFF, 0x1C, 0x1D, 0x1E, 0x1F, 0x85}
    out = [0x20]  # the blank itself (its probe differs: " ?X" alternatives absorb it)
    for c in sorted(cands - {0x20}):
        s = "a" + chr(c) * 2 + "b"
        if [o for _, o in pretok.pre_tokenize_str(s)] == [(0, 1), (1, 2), (2, 3), (3, 4)]:
            out.append(c)
    return out


@functools.lru_cache(maxsize=2)
def _class_table(ws: Tuple[int, ...]) -> bytes:
    cache = Path(os.environ.get("TMPDIR", "/tmp")) / f"smsgate-tokfast-cls-{unicodedata.unidata_version}.bin"
    tab = None
    if cache.exists():
        tab = bytearray(cache.read_bytes())
        if len(tab) != 0x110000:
            tab = None
    if tab is None:
        tab = bytearray(0x110000)
        cat = unicodedata.category
        for c in range(0x110000):
            k = cat(chr(c))
            if k[0] == "L":
                tab[c] = _L
            elif k[0] == "N":
                tab[c] = _N | (_D if k == "Nd" else 0)
        try:
            tmp = cache.with_suffix(f".{os.getpid()}.tmp")
            tmp.write_bytes(bytes(tab))
            os.replace(tmp, cache)
        except OSError:
            pass
    for c in ws:
        tab[c] |= _S
    return bytes(tab)


class FastTokenizer:
    """Batch encode / decode with the native module (same ids as the library)."""

    def __init__(self, tok) -> None:
        ext = _import_ext()
        if ext is None:
            raise ImportError("native tokenizer not built (python -m smsgate_amd.native.build)")
        from .tokenizer import SPECIALS

        self._ext = ext
        self.tok = tok
        spec = json.loads(tok.tk.to_str())
        vocab = spec["model"]["vocab"]
        merges = []
        for m in spec["model"]["merges"]:
            a, b = m if isinstance(m, list) else m.split(" ", 1)
            merges.append((vocab[a], vocab[b], vocab[a + b]))
        specials = [(s.encode(), tok.tk.token_to_id(s)) for s in SPECIALS]
        tb = list(tok.token_bytes)
        ws = tuple(_whitespace(tok.tk.pre_tokenizer))
        self._h = ext.new(tb, merges, _class_table(ws), specials)

    def encode(self, text: str) -> List[int]:
        return self._ext.encode(self._h, text)

    def encode_packed(self, texts: Sequence[str], max_len: int = -1, append_id: int = -1) -> Tuple[int, bytes, bytes]:
        """``(n_truncated, lens: uint16 bytes, ids: int32 bytes)`` -- each text cut to
        ``max_len`` tokens (-1: no cut), then ``append_id`` added (-1: none)."""
        return self._ext.encode_packed(self._h, list(texts), max_len, append_id)

    def decode_fields(self, buf: bytes, offset: int, n: int, nfields: int) -> List[List[str]]:
        """Fields of ``n`` answers packed at ``buf[offset:]`` (lens then ids)."""
        return self._ext.decode_fields(self._h, buf, offset, n, nfields, self.tok.sep)

    def cache_size(self) -> int:
        return self._ext.cache_size(self._h)


@functools.lru_cache(maxsize=4)
def _load(path: str) -> Optional[FastTokenizer]:
    from .tokenizer import load_tokenizer

    try:
        return FastTokenizer(load_tokenizer(path))
    except ImportError:
        return None


def load_fast_tokenizer(path: Optional[str] = None) -> Optional[FastTokenizer]:
    from .tokenizer import ASSET

    if os.environ.get("SMSGATE_NATIVE_TOKENIZER", "1") == "0":
        return None
    return _load(str(path or ASSET))
