"""Synthetic bank-notification SMS with ground-truth fields.

There is no dataset on the box (and the reference ships none — its only
fixtures are the three CASES of tests/test_parsers.py:11-58), so every
benchmark and tokenizer corpus here is generated.  The formats follow the
reference's real-world examples:

* ``APPROVED PURCHASE DB SALE: MERCHANT, CITY[, ADDRESS],dd.mm.yy HH:MM,card ***NNNN. Amount:X CUR, Balance:Y CUR``
  (and the PURCHASE / SALE / PURCHASE DB INTERNET / PURCH.COMPLETION.DB INTERNET prefixes,
  process_cached.py:98-120);
* the multi-line ``DEBIT ACCOUNT&#10;…`` account format (test case 3);
* credit/C2C/OTP/insufficient-funds notifications (worker-skipped kinds).

:func:`generate` is deterministic for a seed.  Each item carries the body and
the expected extraction answer (the LLM JSON shape), so a trained extractor
can be scored and the regex backend cross-checked.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional

__all__ = ["SynthSMS", "generate", "generate_bodies", "reference_cases"]

_WORDS = [
    "TEST", "LLC", "MARKET", "CITY", "CAFE", "PHARMA", "STORE", "YANDEX", "GO", "TAXI", "CARREFOUR", "SAS",
    "ZOVQ", "TASHIR", "PIZZA", "GRAND", "CANDY", "NOR", "ZOV", "WILDBERRIES", "OZON", "AMAZON", "UBER",
    "EATS", "BOLT", "GLOVO", "APPLE", "COM", "BILL", "GOOGLE", "PLAY", "SPOTIFY", "NETFLIX", "STEAM",
    "KFC", "MCDONALDS", "STARBUCKS", "COFFEE", "HOUSE", "BOOKS", "CINEMA", "PARK", "FITNESS", "CLUB",
    "AUTO", "GAS", "STATION", "ELECTRIC", "WATER", "MOBILE", "TELECOM", "VIVA", "UCOM", "TEAM", "BEELINE",
    "AMERIABANK", "API", "GATE", "IDRAM", "EASYPAY", "TELCELL", "POST", "OFFICE", "DUTY", "FREE", "SHOP",
]
_CITIES = ["YEREVAN", "MOSKOW", "AM", "GYUMRI", "VANADZOR", "TBILISI", "DILIJAN", "ONLINE", "LONDON", "DUBAI",
           "PARIS", "BERLIN", "ISTANBUL", "ABOVYAN", "ECHMIADZIN"]
_STREETS = ["TEST STR.", "ABOVYAN STR.", "MASHTOTS AVE.", "TUMANYAN STR.", "KOMITAS AVE.", "SARYAN STR.",
            "BAGHRAMYAN AVE.", "AMIRYAN STR.", "NALBANDYAN STR.", "ARAMI STR."]
_CURRENCIES = ["AMD", "USD", "EUR", "RUB", "GEL"]
_PREFIXES = ["PURCHASE DB SALE", "PURCHASE", "SALE", "PURCHASE DB INTERNET", "PURCH.COMPLETION.DB INTERNET"]


@dataclass
class SynthSMS:
    body: str
    kind: str  # purchase | account | credit | otp | funds
    answer: Optional[Dict[str, Optional[str]]]  # expected LLM JSON answer (None for skipped kinds)
    timestamp: int


def _amount(r: random.Random, cur: str) -> str:
    big = cur in ("AMD", "RUB")
    v = r.uniform(100, 250000) if big else r.uniform(1, 5000)
    s = f"{v:,.2f}" if (big and r.random() < 0.6) else f"{v:.2f}"
    return s


def _merchant(r: random.Random) -> str:
    return " ".join(r.choice(_WORDS) for _ in range(r.choice((1, 1, 2, 2, 3))))


def _address(r: random.Random) -> str:
    a = f"{r.choice(_STREETS)} {r.randint(1, 150)}"
    if r.random() < 0.4:
        a += f", {r.randint(1, 60)} AREA"
    return a


def _date(r: random.Random, year4: bool = False) -> str:
    d, m = r.randint(1, 28), r.randint(1, 12)
    y = r.choice((2023, 2024, 2025))
    hh, mm = r.randint(0, 23), r.randint(0, 59)
    ys = f"{y}" if year4 else f"{y % 100:02d}"
    return f"{d:02d}.{m:02d}.{ys} {hh:02d}:{mm:02d}"


def _one(r: random.Random) -> SynthSMS:
    ts = r.randint(1_690_000_000, 1_750_000_000)
    x = r.random()
    cur = r.choice(_CURRENCIES)
    card = f"{r.randint(0, 9999):04d}"
    if x < 0.55:
        merchant, city = _merchant(r), r.choice(_CITIES)
        address = _address(r) if r.random() < 0.6 else ""
        place = f"{merchant}, {city}" + (f", {address}" if address else "")
        date = _date(r)
        amt, bal = _amount(r, cur), _amount(r, cur)
        pre = r.choice(_PREFIXES)
        status = r.choice(("APPROVED ", "APPROVED ", ""))
        body = f"{status}{pre}: {place},{date},card ***{card}. Amount:{amt} {cur}, Balance:{bal} {cur}"
        ans = dict(txn_type="debit", date=date, amount=amt, currency=cur, card=f"***{card}", merchant=merchant,
                   city=city, address=address, balance=bal)
        return SynthSMS(body, "purchase", ans, ts)
    if x < 0.80:
        merchant, city = _merchant(r), r.choice(_CITIES)
        date = _date(r, year4=True)
        amt, bal = _amount(r, cur), _amount(r, cur)
        first = f"{r.randint(1000, 9999)}"
        body = (f"DEBIT ACCOUNT&#10;{amt} {cur}&#10;{first}***{card},&#10;{merchant}, {city}"
                f"&#10;{date}&#10;BALANCE: {bal} {cur}")
        ans = dict(txn_type="debit", date=date, amount=amt, currency=cur, card=card, merchant=merchant,
                   city=city, address="", balance=bal)
        return SynthSMS(body, "account", ans, ts)
    if x < 0.90:
        kind = r.choice(("CREDIT PAYMENT", "C2C RECEIVED", "TRANSFER IN"))
        date = _date(r)
        amt, bal = _amount(r, cur), _amount(r, cur)
        body = f"{kind}: {date},card ***{card}. Amount:{amt} {cur}, Balance:{bal} {cur}"
        ans = dict(txn_type="credit", date=date, amount=amt, currency=cur, card=f"***{card}", merchant="",
                   city="", address="", balance=bal)
        return SynthSMS(body, "credit", ans, ts)
    if x < 0.96:
        code = r.randint(100000, 999999)
        body = r.choice((f"Your OTP code: {code}. Do not share it.", f"CODE: {code} for login",
                         f"PASS={code} valid 5 min"))
        return SynthSMS(body, "otp", None, ts)
    body = f"DECLINED: INSUFFICIENT FUNDS, {_merchant(r)}, card ***{card}"
    return SynthSMS(body, "funds", None, ts)


def generate(n: int, seed: int = 0, unique: bool = True) -> List[SynthSMS]:
    """``n`` messages; with ``unique`` every body is distinct (defeats the response cache)."""
    r = random.Random(seed)
    out: List[SynthSMS] = []
    seen = set()
    while len(out) < n:
        s = _one(r)
        if unique:
            if s.body in seen:
                continue
            seen.add(s.body)
        out.append(s)
    return out


def generate_bodies(n: int, seed: int = 0) -> List[str]:
    return [s.body for s in generate(n, seed)]


def reference_cases() -> List[str]:
    return [
        "APPROVED PURCHASE DB SALE: TEST LLC, MOSKOW, TEST STR. 29, 24 AREA,06.05.25 14:23,card ***0018. "
        "Amount:52.00 USD, Balance:1842.74 USD",
        "APPROVED PURCHASE DB SALE: TEST, MOSKOW,06.05.25 15:11,card ***0018. Amount:3460.00 USD, "
        "Balance:1800.74 USD",
        "DEBIT ACCOUNT&#10;27,252.00 AMD&#10;4083***7538,&#10;AMERIABANK API GATE, AM&#10;10.06.2025 20:51"
        "&#10;BALANCE: 391,469.09 AMD",
    ]


def iter_corpus(n: int, seed: int = 0) -> Iterator[str]:
    """Tokenizer-training text: bodies, normalised bodies and answer values."""
    from ..parse.text import normalize_body

    for s in generate(n, seed, unique=False):
        yield s.body
        yield normalize_body(s.body)
        if s.answer:
            yield " ".join(v for v in s.answer.values() if v)
