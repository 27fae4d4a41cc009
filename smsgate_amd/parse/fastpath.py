"""The parser processes' native per-message path (``native/csrc/parsefast.cpp``).

VERDICT r05 next #3: host CPU per message dominated the node budget (113.6 us, 8.4x the
GPU's), most of it per-message Python -- RawSMS validation, keyword filters, answer
post-processing, ParsedSMS construction and serialisation.  The extension does that
chain on UTF-8 bytes for the common case and hands every message it cannot prove
equivalent back to the Python path (``None`` from :func:`scan`, :data:`FALLBACK` from
:func:`postprocess`), so the routing and every payload are the Python path's, byte for
byte (tests/test_parsefast.py: the synthetic corpus, hostile strings, the DLQ envelope
shapes).

* :func:`scan` -- sms.raw payloads -> :class:`FastRaw` (a validated RawSMS that no
  keyword filter can touch, with its normalised body and response-cache key) or ``None``;
* :func:`postprocess` -- extractor answer rows (the nine decoded field strings) ->
  the sms.parsed payload bytes, :data:`UNMATCHED` or :data:`FALLBACK`.

``SMSGATE_NATIVE_PARSE=0`` turns it off (the Python path only); :func:`available` is
False when the extension is not built.
"""
from __future__ import annotations

import os
import sys
import unicodedata
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Union

__all__ = ["FastRaw", "available", "scan", "postprocess", "raw_wires", "peek_parsed", "UNMATCHED", "FALLBACK"]

UNMATCHED, FALLBACK = 1, 2
_LIB = Path(__file__).resolve().parent.parent / "native" / "_lib"
_EXT: Any = None
_TRIED = False


class FastRaw:
    """A RawSMS the native scan validated: its native record (``blob``: the UTF-8 fields
    and the pre-encoded sms.parsed fragments), its normalised body (``norm``) and the
    response-cache key of that body (``key`` = parse/cache.py cache_key(norm)).  The
    RawSMS attributes the DLQ envelopes and error reports read (``model_dump`` is
    RawSMS's) are decoded from the record only when asked for."""
    __slots__ = ("blob", "norm", "key", "_f")

    def __init__(self, t) -> None:
        self.blob, self.norm, self.key = t
        self._f = None

    def _fields(self):
        if self._f is None:
            self._f = _EXT.raw_fields(self.blob)
        return self._f

    msg_id = property(lambda self: self._fields()[0])
    sender = property(lambda self: self._fields()[1])
    body = property(lambda self: self._fields()[2])
    date = property(lambda self: self._fields()[3])
    device_id = property(lambda self: self._fields()[4])
    source = property(lambda self: self._fields()[5])

    def model_dump(self) -> Dict[str, Any]:
        f = self._fields()
        return {"msg_id": f[0], "sender": f[1], "body": f[2], "date": f[3], "device_id": f[4], "source": f[5]}


def _tables():
    """(chars whose upper case contains an ASCII letter, non-ASCII \\d digits, currency
    alias variants whose .upper() is the alias key)."""
    from .canonical import CURRENCY_ALIASES

    upper, digits = [], []
    for c in range(0x80, 0x110000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        ch = chr(c)
        if any(ord(x) < 0x80 for x in ch.upper()):
            upper.append(ch)
        if unicodedata.category(ch) == "Nd":
            digits.append(ch)
    aliases: Dict[str, str] = {}
    for key, code in CURRENCY_ALIASES.items():
        for v in {key, key.lower(), key.title(), key.capitalize(), key.casefold()}:
            if v.upper() == key:
                aliases[v] = code
    return "".join(upper), "".join(digits), aliases


def _ext():
    global _EXT, _TRIED
    if _TRIED:
        return _EXT
    _TRIED = True
    if os.environ.get("SMSGATE_NATIVE_PARSE", "1") == "0":
        return None
    p = str(_LIB)
    if p not in sys.path:
        sys.path.insert(0, p)
    try:
        import _parsefast  # type: ignore
    except ImportError:
        return None
    _parsefast.init(*_tables())
    _EXT = _parsefast
    return _EXT


def available() -> bool:
    return _ext() is not None


def _now():
    n = datetime.now()
    return (n.year, n.month, n.day, n.hour, n.minute, n.second, n.microsecond)


def scan(payloads: Sequence[bytes]) -> List[Optional[FastRaw]]:
    """Per sms.raw payload: a :class:`FastRaw`, or None (the Python path decides)."""
    ext = _ext()
    if ext is None:
        return [None] * len(payloads)
    return [None if t is None else FastRaw(t) for t in ext.scan_raw(payloads)]


def postprocess(rows: List[List[str]], raws: Sequence[FastRaw]) -> List[Union[bytes, int]]:
    """Per answer row (txn_type, date, amount, currency, card, merchant, city, address,
    balance -- decoded strings): the sms.parsed payload, UNMATCHED or FALLBACK."""
    ext = _ext()
    if ext is None:
        return [FALLBACK] * len(rows)
    return ext.postprocess(rows, [r.blob for r in raws], _now())


def raw_wires(payloads) -> List[bytes]:
    """``raw_wire(payload_to_raw(p))`` of gateway payloads (services/gateway.py
    RawSMSPayload): the md5 message id and RawSMS's JSON natively, the Python path for
    any payload RawSMS validation would refuse (it raises there)."""
    from ..models.domain import raw_wire
    from ..services.gateway import payload_to_raw

    ext = _ext()
    got = ext.raw_wires([(p.device_id, p.message, p.sender, p.timestamp, p.source) for p in payloads]) \
        if ext is not None else [None] * len(payloads)
    return [g if g is not None else raw_wire(payload_to_raw(p)) for g, p in zip(got, payloads)]


def peek_parsed(payloads: Sequence[bytes]) -> List[Optional[tuple]]:
    """The writer's check of sms.parsed payloads: per payload ``(msg_id, merchant is
    truthy, (y, mo, d, h, mi, s))`` when it is the canonical form of a valid ParsedSMS
    (every field checked natively), else None (pydantic decides)."""
    ext = _ext()
    if ext is None:
        return [None] * len(payloads)
    return ext.peek_parsed(payloads)
