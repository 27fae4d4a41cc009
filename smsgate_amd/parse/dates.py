"""Date/time normalisation chain of the parse pipeline.

Behaviour-compatible with the reference helpers (golden-tested):

* :func:`parse_custom_datetime` — ``'%d.%m.%y %H:%M'`` first, then a free-form
  ``dateutil`` parse (gemini_parser.py:106-119).
* :func:`parse_unix_timestamp` — seconds vs milliseconds auto-detection
  (< 1e11 s, < 1e14 ms), conversion into an IANA zone, optionally naive
  (gemini_parser.py:139-188).
* :func:`fix_broken_datetime` — the first ``dd.mm.yyyy`` (else ``dd.mm.yy``)
  date found in the SMS body overrides the *date part* of the LLM's answer
  while its time of day is kept (gemini_parser.py:67-104). This repairs
  day/month swaps made by the model.
"""
from __future__ import annotations

import re
import zoneinfo
from datetime import datetime, timezone
from typing import Union

from dateutil.parser import parse as _du_parse

__all__ = [
    "parse_custom_datetime",
    "parse_unix_timestamp",
    "fix_broken_datetime",
    "TimestampParseError",
]

_BODY_DATE_PATTERNS = (
    (re.compile(r"\d{2}\.\d{2}\.\d{4}"), "%d.%m.%Y"),
    (re.compile(r"\d{2}\.\d{2}\.\d{2}"), "%d.%m.%y"),
)


class TimestampParseError(ValueError):
    """Raised for values that cannot be a Unix timestamp."""


# ``strptime`` costs ~18 µs per call and ran twice per message on the hot path.
# Exact-shape inputs take an integer fast path with identical results
# (including ValueError for impossible dates and POSIX %y pivoting:
# 69–99 → 19xx, 00–68 → 20xx); everything else goes through strptime/dateutil.
_FAST_DMY_HM = re.compile(r"(\d\d)\.(\d\d)\.(\d\d) (\d\d):(\d\d)\Z")


def _yy(y: int) -> int:
    return y + (1900 if y >= 69 else 2000)


# ``dateutil`` costs ~75 us per call, and every layout but the reference's dd.mm.yy
# HH:MM reaches it.  The shapes below are computed directly, with dateutil's own
# resolution rules (a dotted d.m.y is read MONTH first when it can be -- the body-date
# repair fixes the date part afterwards -- 2-digit years via its century window, English
# month abbreviations); any value the fast path cannot build (an impossible date) falls
# through to dateutil, so errors are dateutil's own.  tests/test_parse_helpers.py fuzzes
# every shape against dateutil.
_FAST_ISO = re.compile(r"(\d{4})-(\d{2})-(\d{2})(?:[ T](\d{2}):(\d{2})(?::(\d{2}))?)?\Z")
_FAST_DOTTED = re.compile(r"(\d{2})\.(\d{2})\.(\d{4}|\d{2})(?: (\d{2}):(\d{2}))?\Z")
_FAST_TIME_FIRST = re.compile(r"(\d{2}):(\d{2}) (\d{2})\.(\d{2})\.(\d{4})\Z")
_FAST_MON = re.compile(r"(\d{1,2})([ -])([A-Za-z]{3})\2(\d{4})(?: (\d{2}):(\d{2}))?\Z")
_MONTHS = {m: i for i, m in enumerate(("jan", "feb", "mar", "apr", "may", "jun", "jul", "aug", "sep", "oct", "nov",
                                       "dec"), 1)}
# dateutil's month words (parserinfo.MONTHS: abbreviation, "Sept", full name; any case)
_MONTH_WORDS = {**_MONTHS, **{w: i for i, w in enumerate(("january", "february", "march", "april", "may", "june",
                                                          "july", "august", "september", "october", "november",
                                                          "december"), 1)}, "sept": 9}
# the value grammar's other shapes (12-hour clocks, month names; round 6): each computed
# with dateutil's rules -- a dotted d.m.y month first when it can be, "12 AM" = 0 h,
# "h PM" = h + 12, an hour over 12 with AM / PM is dateutil's error (falls through)
_AMPM = r"(?: ?([AaPp][Mm]))"
_FAST_ISO_12 = re.compile(r"(\d{4})-(\d{2})-(\d{2}) (\d{1,2}):(\d{2})" + _AMPM + r"\Z")
_FAST_DOTTED_12 = re.compile(r"(\d{2})\.(\d{2})\.(\d{4}) (\d{1,2}):(\d{2})" + _AMPM + r"\Z")
_FAST_TIME_FIRST_12 = re.compile(r"(\d{1,2}):(\d{2})" + _AMPM + r" (\d{2})\.(\d{2})\.(\d{4})\Z")
_FAST_MDY = re.compile(r"([A-Za-z]{3,9}) (\d{1,2}), (\d{4})(?: (\d{1,2}):(\d{2})" + _AMPM + r"?)?\Z")
_FAST_DMY_WORD = re.compile(r"(\d{1,2}) ([A-Za-z]{3,9}) (\d{4})(?: (\d{1,2}):(\d{2})" + _AMPM + r"?)?\Z")
_DU_INFO = None


def _du_year(y: int) -> int:
    global _DU_INFO
    if _DU_INFO is None:
        from dateutil.parser import parserinfo

        _DU_INFO = parserinfo()
    return _DU_INFO.convertyear(y)


def _month_first(a: int, b: int, y: int, hh: int = 0, mm: int = 0) -> datetime:
    """dateutil's reading of an all-numeric d.m.y: month first unless it cannot be."""
    if a <= 12:
        return datetime(y, a, b, hh, mm)
    return datetime(y, b, a, hh, mm)


def _hour12(h: int, ampm) -> int:
    """dateutil's AM / PM rule (None: a 24-hour time); -1 for an hour it refuses."""
    if ampm is None:
        return h
    if not 0 <= h <= 12:
        return -1
    pm = ampm[0] in "Pp"
    return h + 12 if (pm and h < 12) else 0 if (not pm and h == 12) else h


def _fast_dateutil_12(text: str):
    m = _FAST_ISO_12.match(text)
    if m is not None:
        y, mo, d, hh, mi, ap = m.groups()
        h = _hour12(int(hh), ap)
        return None if h < 0 else datetime(int(y), int(mo), int(d), h, int(mi))
    m = _FAST_DOTTED_12.match(text)
    if m is not None:
        a, b, y, hh, mi, ap = m.groups()
        h = _hour12(int(hh), ap)
        return None if h < 0 else _month_first(int(a), int(b), int(y), h, int(mi))
    m = _FAST_TIME_FIRST_12.match(text)
    if m is not None:
        hh, mi, ap, a, b, y = m.groups()
        h = _hour12(int(hh), ap)
        return None if h < 0 else _month_first(int(a), int(b), int(y), h, int(mi))
    m = _FAST_MDY.match(text) or _FAST_DMY_WORD.match(text)
    if m is not None:
        if m.re is _FAST_MDY:
            word, d, y, hh, mi, ap = m.groups()
        else:
            d, word, y, hh, mi, ap = m.groups()
        mo = _MONTH_WORDS.get(word.lower())
        if mo is None:
            return None
        h = _hour12(int(hh), ap) if hh is not None else 0
        return None if h < 0 else datetime(int(y), mo, int(d), h, int(mi or 0))
    return None


def _fast_dateutil(text: str):
    try:
        m = _FAST_ISO.match(text)
        if m is not None:
            y, mo, d, hh, mi, ss = m.groups()
            return datetime(int(y), int(mo), int(d), int(hh or 0), int(mi or 0), int(ss or 0))
        m = _FAST_DOTTED.match(text)
        if m is not None:
            a, b, y, hh, mi = m.groups()
            yy = int(y) if len(y) == 4 else _du_year(int(y))
            return _month_first(int(a), int(b), yy, int(hh or 0), int(mi or 0))
        m = _FAST_TIME_FIRST.match(text)
        if m is not None:
            hh, mi, a, b, y = map(int, m.groups())
            return _month_first(a, b, y, hh, mi)
        m = _FAST_MON.match(text)
        if m is not None:
            d, _, mon, y, hh, mi = m.groups()
            mo = _MONTHS.get(mon.lower())
            if mo is not None:
                return datetime(int(y), mo, int(d), int(hh or 0), int(mi or 0))
        if text[-1:] in "MmrRyYlLtTeEnNhHvV0123456789":  # (cheap pre-check: AM / PM or a month word / digit last)
            return _fast_dateutil_12(text)
    except ValueError:
        return None  # impossible date: dateutil decides (and raises its own error)
    return None


def parse_custom_datetime(text: str) -> datetime:
    if isinstance(text, str):
        m = _FAST_DMY_HM.match(text)
        if m is not None:
            d, mo, y, hh, mm = map(int, m.groups())
            try:
                return datetime(_yy(y), mo, d, hh, mm)
            except ValueError:
                pass  # impossible date: same fallback path as strptime's failure
        else:
            fast = _fast_dateutil(text)  # shapes strptime('%d.%m.%y %H:%M') always rejects
            if fast is not None:
                return fast
    try:
        return datetime.strptime(text, "%d.%m.%y %H:%M")
    except Exception:
        dt = _du_parse(text)
    if dt.tzinfo is not None:
        # a numeric zone of a day or more ("10:00 +2500") builds an aware datetime whose
        # every later use -- printing, comparing, converting -- raises; raise here, where
        # a parse error is a parse failure (the message is dead-lettered, not its batch)
        dt.utcoffset()
    return dt


def parse_unix_timestamp(ts: Union[int, float, str], tz: str = "UTC", aware: bool = True) -> datetime:
    try:
        num = float(ts)
    except (TypeError, ValueError):
        raise TimestampParseError(f"unsupported timestamp {ts!r}") from None
    if num < 0:
        raise TimestampParseError("negative timestamps are not supported")
    if num < 1e11:
        seconds = num
    elif num < 1e14:
        seconds = num / 1000.0
    else:
        raise TimestampParseError("value does not look like a Unix timestamp in s or ms")
    local = datetime.fromtimestamp(seconds, tz=timezone.utc).astimezone(zoneinfo.ZoneInfo(tz))
    return local if aware else local.replace(tzinfo=None)


def _date_from_match(s: str, fmt: str) -> datetime:
    # the regexes guarantee dd.mm.yyyy / dd.mm.yy shapes, so this equals strptime
    d, mo, y = int(s[0:2]), int(s[3:5]), int(s[6:])
    return datetime(y if fmt == "%d.%m.%Y" else _yy(y), mo, d)


def fix_broken_datetime(body: str, current: datetime) -> datetime:
    # every dd.mm.yyyy match is also a dd.mm.yy match starting at the same place, so the
    # first dd.mm.yy match bounds where a dd.mm.yyyy one can start: one full scan of the
    # body instead of up to two (same precedence as the reference's loop)
    (rx4, fmt4), (rx2, fmt2) = _BODY_DATE_PATTERNS
    m2 = rx2.search(body)
    if m2 is None:
        return current
    for m, fmt in ((rx4.search(body, m2.start()), fmt4), (m2, fmt2)):
        if m is None:
            continue
        try:
            day = _date_from_match(m.group(0), fmt)
        except ValueError:
            continue
        # ``time()`` drops tzinfo, exactly like the reference: a repaired date
        # is naive local time.
        return datetime.combine(day.date(), current.time())
    return current
