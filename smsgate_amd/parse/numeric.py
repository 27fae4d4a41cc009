"""Locale-agnostic amount parsing.

Behaviour-compatible with ``parse_ambiguous_decimal`` (libs/decimal_utils.py:4-63),
including its documented quirks, which are *contracts* (golden tests in
``tests/test_parse_helpers.py``):

* the right-most of ``.``/``,`` is the decimal mark when both occur;
* a single ``,`` is a decimal mark (``'1,000' -> 1.000``), several are
  thousands separators;
* several ``.``: all but the last are thousands separators
  (``'1.234.567' -> 1234.567``);
* blanks are dropped, then everything but ``[0-9.-]``; empty -> ``0.0``;
* an unparsable remainder (e.g. ``'None'``) raises :class:`ValueError`.
"""
from __future__ import annotations

import re
from decimal import Decimal, InvalidOperation
from typing import Union

__all__ = ["parse_ambiguous_decimal"]

_KEEP = re.compile(r"[^0-9.\-]")


def _canonical(s: str) -> str:
    dot, comma = s.rfind("."), s.rfind(",")
    if dot >= 0 and comma >= 0:
        # Both marks present: whichever comes last is the decimal mark.
        if comma > dot:
            return s.replace(".", "").replace(",", ".")
        return s.replace(",", "")
    if comma >= 0:
        return s.replace(",", "") if s.count(",") > 1 else s.replace(",", ".")
    if dot >= 0 and s.count(".") > 1:
        head, _, tail = s.rpartition(".")
        return head.replace(".", "") + "." + tail
    return s


def parse_ambiguous_decimal(value: Union[str, int, float, Decimal]) -> Decimal:
    """Parse an amount written in an unknown locale into a :class:`Decimal`."""
    if not isinstance(value, str):
        return Decimal(value)
    s = value.strip().replace(" ", "")
    if not s:
        return Decimal("0.0")
    canon = _KEEP.sub("", _canonical(s))
    try:
        return Decimal(canon)
    except InvalidOperation:
        raise ValueError(f"cannot parse amount {value!r} (cleaned to {canon!r})") from None
