"""Offline rule-based extractor with the LLM's answer shape.

The reference's pre-LLM parser (``process_cached.py:98-204``) handled two
single-line formats, put the city into ``address`` and returned ``None`` for the
multi-line ``DEBIT ACCOUNT`` format.  This backend is a clean
re-design that returns the *same string-valued JSON an LLM returns*, so it goes
through the identical post-processing chain, and covers:

* single-line card purchases:
  ``[APPROVED|REVERSE…] <PURCHASE|SALE|PURCHASE DB SALE|PURCHASE DB INTERNET|
  PURCH.COMPLETION.DB INTERNET>: MERCHANT, CITY[, ADDRESS…],dd.mm.yy HH:MM,card ***NNNN.
  Amount:X CUR, Balance:Y CUR``;
* single-line credits: ``<TYPE>: dd.mm.yy HH:MM,card ***NNNN. Amount:X CUR, Balance:Y CUR``;
* multi-line account notifications (real newlines or the ``&#10;`` entity
  of XML backups): ``DEBIT|CREDIT ACCOUNT / amount CUR / card / MERCHANT, CITY /
  date / BALANCE: Y CUR``.

Anything else yields :data:`UNKNOWN_ANSWER` (``txn_type="unknown"``, all
fields null), which post-processing rejects → DLQ ``unmatched``, the same
route an LLM "nothing found" answer takes.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Sequence

from .base import ExtractResult, ParserBackend

__all__ = ["RegexBackend", "extract_rule_based", "UNKNOWN_ANSWER"]

UNKNOWN_ANSWER: Dict[str, Any] = {
    "txn_type": "unknown", "date": None, "amount": None, "currency": None, "card": None,
    "merchant": None, "city": None, "address": None, "balance": None,
}

_NUM = r"[\d][\d.,\s]*"
_DATE = r"\d{2}[./-]\d{2}[./-]\d{2,4}\s+\d{2}:\d{2}"

_PURCHASE = re.compile(
    r"(?P<kind>PURCHASE\s+DB\s+INTERNET|PURCH\.COMPLETION\.DB\s+INTERNET|PURCHASE\s+DB\s+SALE|PURCHASE|SALE)"
    r"\s*:\s*(?P<place>.*?)\s*,\s*(?P<date>" + _DATE + r")\s*,\s*card\s+(?P<card>[*\d]+)\s*\.\s*"
    r"Amount\s*:\s*(?P<amount>" + _NUM + r"?)\s*(?P<cur>[A-Z]{3})\s*,\s*"
    r"Balance\s*:\s*(?P<bal>" + _NUM + r"?)\s*(?P<bcur>[A-Z]{3})",
    re.I | re.S,
)
_CREDIT = re.compile(
    r"(?P<kind>[A-Z][A-Z0-9 ]*?)\s*:\s*(?P<date>" + _DATE + r")\s*,\s*card\s+(?P<card>[*\d]+)\s*\.\s*"
    r"Amount\s*:\s*(?P<amount>" + _NUM + r"?)\s*(?P<cur>[A-Z]{3})\s*,\s*"
    r"Balance\s*:\s*(?P<bal>" + _NUM + r"?)\s*(?P<bcur>[A-Z]{3})",
    re.I | re.S,
)
_LINES = re.compile(r"&#10;|\r?\n")
_AMOUNT_LINE = re.compile(r"^(?P<amount>" + _NUM + r"?)\s*(?P<cur>[A-Z]{3})$")
_CARD_LINE = re.compile(r"^(?:CARD:(?P<c1>\d{4})|[*\d]*\*+(?P<c2>\d{4})),?$", re.I)
_DATE_LINE = re.compile(r"^(?P<date>" + _DATE + r")$")
_BAL_LINE = re.compile(r"^BALANCE\s*:\s*(?P<bal>" + _NUM + r"?)\s*(?P<cur>[A-Z]{3})$", re.I)


def _split_place(place: str) -> Dict[str, str]:
    parts = [p.strip() for p in place.split(",")]
    merchant = parts[0] if parts else ""
    city = parts[1] if len(parts) > 1 else ""
    address = ", ".join(p for p in parts[2:]) if len(parts) > 2 else ""
    return {"merchant": merchant, "city": city, "address": address}


def _multiline(body: str) -> Optional[Dict[str, Any]]:
    lines = [ln.strip() for ln in _LINES.split(body) if ln.strip()]
    if len(lines) < 4:
        return None
    head = lines[0].upper()
    if "DEBIT" in head:
        txn = "debit"
    elif "CREDIT" in head:
        txn = "credit"
    else:
        return None
    out: Dict[str, Any] = {"txn_type": txn, "merchant": "", "city": "", "address": ""}
    for ln in lines[1:]:
        if "amount" not in out and (m := _AMOUNT_LINE.match(ln)):
            out["amount"], out["currency"] = m.group("amount").strip(), m.group("cur").upper()
        elif "card" not in out and (m := _CARD_LINE.match(ln)):
            out["card"] = m.group("c1") or m.group("c2")
        elif "date" not in out and (m := _DATE_LINE.match(ln)):
            out["date"] = m.group("date")
        elif "balance" not in out and (m := _BAL_LINE.match(ln)):
            out["balance"] = m.group("bal").strip()
        elif not out["merchant"] and "," in ln:
            out.update(_split_place(ln))
    if not {"amount", "date"} <= out.keys():
        return None
    out.setdefault("card", None)
    out.setdefault("balance", None)
    out.setdefault("currency", None)
    return out


def extract_rule_based(body: str) -> Optional[Dict[str, Any]]:
    """Return the LLM-shaped answer for a known format, else ``None``."""
    m = _PURCHASE.search(body)
    if m:
        ans = {
            "txn_type": "debit",
            "date": m.group("date"),
            "amount": m.group("amount").strip(),
            "currency": m.group("cur").upper(),
            "card": m.group("card"),
            "balance": m.group("bal").strip(),
        }
        ans.update(_split_place(m.group("place")))
        return ans
    ml = _multiline(body)
    if ml is not None:
        return ml
    m = _CREDIT.search(body)
    if m:
        return {
            "txn_type": "credit",
            "date": m.group("date"),
            "amount": m.group("amount").strip(),
            "currency": m.group("cur").upper(),
            "card": m.group("card"),
            "merchant": "",
            "city": "",
            "address": "",
            "balance": m.group("bal").strip(),
        }
    return None


class RegexBackend(ParserBackend):
    name = "regex"
    max_batch = 1024

    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        out: List[ExtractResult] = []
        for b in bodies:
            ans = extract_rule_based(b)
            # Unknown format: answer like an LLM that found nothing — the
            # post-processing chain then routes it to the DLQ as "unmatched".
            out.append(ans if ans is not None else dict(UNKNOWN_ANSWER))
        return out
