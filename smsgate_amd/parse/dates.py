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


def parse_custom_datetime(text: str) -> datetime:
    if isinstance(text, str):
        m = _FAST_DMY_HM.match(text)
        if m is not None:
            d, mo, y, hh, mm = map(int, m.groups())
            try:
                return datetime(_yy(y), mo, d, hh, mm)
            except ValueError:
                pass  # impossible date: same fallback path as strptime's failure
    try:
        return datetime.strptime(text, "%d.%m.%y %H:%M")
    except Exception:
        return _du_parse(text)


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
