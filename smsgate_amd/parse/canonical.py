"""Answer canonicalisation for copy-span extractors (runs before post-processing).

The reference asks Gemini for strings and lets post-processing parse them
(gemini_parser.py:224-241); a hosted LLM quietly normalises as it answers
(``$`` -> ``USD``).  The local extractor *copies* every value from the body
(serving/fsm.py copy constraint), so a value can be a currency symbol or a
date in a layout the reference chain mis-reads.  Two deterministic fixes, applied
to every backend's answer by :func:`~smsgate_amd.parse.pipeline.postprocess_answer`:

* **currency**: a symbol or word (``$ € ֏ ₽ ₾ £``, ``руб``, ``драм``…) becomes its
  ISO 4217 code; codes pass through unchanged (ParsedSMS upper-cases them);
* **day-first numeric dates with ``/`` or ``-``** (``06/05/2025 14:23``,
  ``06-05-25``) become ISO ``2025-05-06 14:23``.  ``dateutil`` reads them
  month-first, and the reference's body-date repair (``fix_broken_datetime``)
  only knows dotted dates, so without this a ``dd/mm/yyyy`` SMS would be stored
  with day and month swapped.  Day-first is the reference's own convention
  (SYSTEM_INSTRUCTION: "Дата в сообщении обычно в формате день.месяц.год").
  Dotted dates are left to the reference chain (its golden behaviour).

Values that are not strings (a ``None`` from an LLM) pass through untouched, so
D6 / D8 (null amount / card -> DLQ) stay as they were.
"""
from __future__ import annotations

import re
from typing import Any, Dict

__all__ = ["CURRENCY_ALIASES", "canonical_currency", "canonical_date_text", "canonicalize_answer"]

CURRENCY_ALIASES: Dict[str, str] = {
    "$": "USD", "US$": "USD", "€": "EUR", "EURO": "EUR", "֏": "AMD", "ДРАМ": "AMD", "DRAM": "AMD",
    "₽": "RUB", "РУБ": "RUB", "Р": "RUB", "RUR": "RUB", "₾": "GEL", "£": "GBP",
}

_DAY_FIRST = re.compile(r"(\d{1,2})[/-](\d{1,2})[/-](\d{4}|\d{2})(?![\d])(.*)\Z", re.S)
# Russian month names (genitive, "6 июня 2025 14:23"; also the nominative / short forms,
# "г." / "в" before the time of day, the time first, and Latin transliterations):
# dateutil knows English month names only, so without this the date would fall back to
# the message timestamp
_RU_MONTHS = {"январ": 1, "феврал": 2, "март": 3, "апрел": 4, "ма": 5, "июн": 6, "июл": 7, "август": 8,
              "сентябр": 9, "октябр": 10, "ноябр": 11, "декабр": 12}
_RU_DATE = re.compile(r"(\d{1,2})\s+([а-яё]+)\.?\s+(\d{4})(?:\s*г\.?)?(?:\s+в(?=\s))?(.*)\Z", re.S | re.I)
# the time of day first: "14:23 6 июня 2025" (and the transliterated "14:23 6 iyunya 2025")
_MONTH_TIME_FIRST = re.compile(r"(\d{1,2}:\d{2}(?::\d{2})?)\s+(\d{1,2})\s+([^\W\d_]+)\.?\s+(\d{4})(?:\s*г\.?)?\Z",
                               re.I)
_RU_ENDINGS = ("я", "а", "ь", "й", "е", "")
# Russian month names in Latin letters (the transliterated SMS: "6 iyunya 2025 14:23")
_TR_MONTHS = {w: i for i, ws in enumerate((
    ("yanvarya", "yanvar"), ("fevralya", "fevral"), ("marta", "mart"), ("aprelya", "aprel"), ("maya", "mai"),
    ("iyunya", "iyun"), ("iyulya", "iyul"), ("avgusta", "avgust"), ("sentyabrya", "sentyabr"),
    ("oktyabrya", "oktyabr"), ("noyabrya", "noyabr"), ("dekabrya", "dekabr")), 1) for w in ws}
_TR_DATE = re.compile(r"(\d{1,2})\s+([a-z]+)\s+(\d{4})(?:\s*g\.?)?(?:\s+v(?=\s))?(.*)\Z", re.S | re.I)


def _ru_month(word: str) -> int:
    w = word.lower()
    for end in _RU_ENDINGS:
        if end and not w.endswith(end):
            continue
        stem = w[: len(w) - len(end)] if end else w
        if stem in _RU_MONTHS:
            return _RU_MONTHS[stem]
        if len(stem) >= 3:  # "сент", "окт"
            hits = [m for s, m in _RU_MONTHS.items() if len(s) >= 3 and s.startswith(stem)]
            if len(hits) == 1:
                return hits[0]
    return 0


def canonical_currency(value: Any) -> Any:
    if not isinstance(value, str):
        return value
    v = value.strip().rstrip(".")
    return CURRENCY_ALIASES.get(v.upper(), value)


def _month_number(word: str) -> int:
    """Month of a Russian (Cyrillic) or transliterated month name, 0 for anything else
    (English names are dateutil's)."""
    return _ru_month(word) if not word.isascii() else _TR_MONTHS.get(word.lower(), 0)


def canonical_date_text(value: Any) -> Any:
    if not isinstance(value, str):
        return value
    v = value.strip()
    m = _DAY_FIRST.match(v)
    if m is None:
        t = _MONTH_TIME_FIRST.match(v)
        if t is not None:
            mo, d = _month_number(t.group(3)), int(t.group(2))
            if mo and 1 <= d <= 31:
                return f"{t.group(4)}-{mo:02d}-{d:02d} {t.group(1)}"
            return value
        r = _RU_DATE.match(v) if not v.isascii() else _TR_DATE.match(v)
        if r is not None:
            mo = _month_number(r.group(2))
            d = int(r.group(1))
            if mo and 1 <= d <= 31:
                return f"{r.group(3)}-{mo:02d}-{d:02d}{r.group(4)}"
        return value
    d, mo, y, rest = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)
    if not (1 <= d <= 31 and 1 <= mo <= 12):
        return value
    year = int(y) if len(y) == 4 else 2000 + int(y) if int(y) < 69 else 1900 + int(y)
    return f"{year:04d}-{mo:02d}-{d:02d}{rest}"


def canonicalize_answer(answer: Dict[str, Any]) -> Dict[str, Any]:
    """A copy of ``answer`` with currency and date canonicalised (see module doc)."""
    out = dict(answer)
    if "currency" in out:
        out["currency"] = canonical_currency(out["currency"])
    if "date" in out:
        out["date"] = canonical_date_text(out["date"])
    return out
