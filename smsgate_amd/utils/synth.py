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
import zlib
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

__all__ = ["SynthSMS", "generate", "generate_bodies", "reference_cases", "vocab", "Vocab", "TRAFFIC_KINDS"]

# Real-looking merchant words.  The reference's golden answers (tests/test_parsers.py:11-58:
# TEST, LLC, MOSKOW, AMERIABANK, API, GATE, AM, "TEST STR.") are deliberately absent from
# every pool, so the three golden CASES are out-of-vocabulary for a model trained here.
_GOLDEN_VOCAB = frozenset({"TEST", "LLC", "MOSKOW", "AMERIABANK", "API", "GATE", "AM"})
_REAL_WORDS = [
    "MARKET", "CITY", "CAFE", "PHARMA", "STORE", "YANDEX", "GO", "TAXI", "CARREFOUR", "SAS",
    "ZOVQ", "TASHIR", "PIZZA", "GRAND", "CANDY", "NOR", "ZOV", "WILDBERRIES", "OZON", "AMAZON", "UBER",
    "EATS", "BOLT", "GLOVO", "APPLE", "COM", "BILL", "GOOGLE", "PLAY", "SPOTIFY", "NETFLIX", "STEAM",
    "KFC", "MCDONALDS", "STARBUCKS", "COFFEE", "HOUSE", "BOOKS", "CINEMA", "PARK", "FITNESS", "CLUB",
    "AUTO", "GAS", "STATION", "ELECTRIC", "WATER", "MOBILE", "TELECOM", "VIVA", "UCOM", "TEAM", "BEELINE",
    "IDRAM", "EASYPAY", "TELCELL", "POST", "OFFICE", "DUTY", "FREE", "SHOP", "INC", "LTD", "CJSC", "OJSC",
    "BANK", "PAY", "ONLINE", "EXPRESS", "CENTER", "MALL", "FOOD", "BAR", "GRILL", "HOTEL", "TRAVEL", "AIR",
]
_REAL_CITIES = ["YEREVAN", "GYUMRI", "VANADZOR", "TBILISI", "DILIJAN", "ONLINE", "LONDON", "DUBAI", "PARIS",
                "BERLIN", "ISTANBUL", "ABOVYAN", "ECHMIADZIN", "MOSCOW", "KAPAN", "BATUMI", "RIGA", "PRAGUE"]
_STREET_SUFFIXES = ["STR.", "AVE.", "ST.", "BLVD", "SQ.", "LANE"]
_CURRENCIES = ["AMD", "USD", "EUR", "RUB", "GEL"]
_PREFIXES = ["PURCHASE DB SALE", "PURCHASE", "SALE", "PURCHASE DB INTERNET", "PURCH.COMPLETION.DB INTERNET"]

_ONSETS = ["B", "D", "G", "K", "L", "M", "N", "P", "R", "S", "T", "V", "Z", "KH", "SH", "TS", "GR", "ST",
           "BR", "DR", "KR", "TR", "CH", "Y", "H", "F"]
_VOWELS = ["A", "E", "I", "O", "U", "YA", "OU", "EA", "IO"]
_CODAS = ["", "", "", "N", "R", "S", "K", "T", "M", "L", "RT", "NK"]


def _pseudo_words(seed: int = 20240601, n: int = 20000, exclude=frozenset()) -> List[str]:
    """``n`` pronounceable capitalised pseudo-words, deterministic for ``seed``."""
    r = random.Random(seed)
    seen = set(exclude)
    out: List[str] = []
    while len(out) < n:
        w = "".join(r.choice(_ONSETS) + r.choice(_VOWELS) + r.choice(_CODAS) for _ in range(r.choice((1, 2, 2, 3))))
        if 2 <= len(w) <= 12 and w not in seen and w not in _GOLDEN_VOCAB:
            seen.add(w)
            out.append(w)
    return out


def _random_strings(seed: int = 99, n: int = 6000) -> List[str]:
    """Letter/digit strings with no syllable structure: a language model cannot
    predict them, so the extractor has to learn to *copy* names from the body."""
    r = random.Random(seed)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZ"
    out: List[str] = []
    seen = set(_GOLDEN_VOCAB)
    while len(out) < n:
        k = r.randint(2, 10)
        w = "".join(r.choice(alpha if r.random() < 0.9 else "0123456789") for _ in range(k))
        if w[0].isalpha() and w not in seen:
            seen.add(w)
            out.append(w)
    return out


def _split(words: Sequence[str]) -> Tuple[List[str], List[str]]:
    """Deterministic train / held-out split (crc32 % 5 == 0 -> held out)."""
    tr, ho = [], []
    for w in words:
        (ho if zlib.crc32(w.encode()) % 5 == 0 else tr).append(w)
    return tr, ho


@dataclass(frozen=True)
class Vocab:
    """Word pools one generator draws merchants / cities / streets from."""
    words: Tuple[str, ...]
    cities: Tuple[str, ...]
    streets: Tuple[str, ...]


def _vocabs() -> Dict[str, Vocab]:
    pw = _pseudo_words()
    pw_tr, pw_ho = _split(pw)
    rs_tr, rs_ho = _split(_random_strings())
    # a third, disjoint pseudo-word pool for the tokenizer's corpus only: it learns
    # syllable-level pieces without any train / held-out / golden word becoming a token
    pw_tok = _pseudo_words(seed=777, n=20000, exclude=frozenset(pw) | _GOLDEN_VOCAB)
    rw_tr, rw_ho = _split(_REAL_WORDS)
    rc_tr, rc_ho = _split(_REAL_CITIES)
    half_tr, half_ho = len(pw_tr) // 2, len(pw_ho) // 2
    return {
        # merchants mix real and pseudo words; cities / streets are mostly pseudo names
        "train": Vocab(tuple(rw_tr * 20 + pw_tr[:half_tr] + rs_tr), tuple(rc_tr * 40 + pw_tr[half_tr:] + rs_tr),
                       tuple(pw_tr[half_tr:] + rs_tr)),
        "heldout": Vocab(tuple(rw_ho * 20 + pw_ho[:half_ho] + rs_ho), tuple(rc_ho * 40 + pw_ho[half_ho:] + rs_ho),
                         tuple(pw_ho[half_ho:] + rs_ho)),
        # the tokenizer's corpus: real training-split words plus the separate pseudo-word
        # pool, so no train / held-out / golden-case word is itself a merged token —
        # all of them split into the same kind of syllable pieces
        "tokenizer": Vocab(tuple(rw_tr * 20 + pw_tok[:10000]), tuple(rc_tr * 40 + pw_tok[10000:]),
                           tuple(pw_tok[10000:])),
    }


_VOCABS: Dict[str, Vocab] = {}


def vocab(name: str = "train") -> Vocab:
    if not _VOCABS:
        _VOCABS.update(_vocabs())
    return _VOCABS[name]


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


def _merchant(r: random.Random, v: Vocab) -> str:
    m = " ".join(r.choice(v.words) for _ in range(r.choice((1, 1, 2, 2, 3, 4))))
    if r.random() < 0.08:
        m += f" {r.randint(1, 999)}"
    return m


def _address(r: random.Random, v: Vocab) -> str:
    a = f"{r.choice(v.streets)} {r.choice(_STREET_SUFFIXES)} {r.randint(1, 150)}"
    if r.random() < 0.4:
        a += f", {r.randint(1, 60)} AREA"
    return a


def _date(r: random.Random, year4: bool = False) -> str:
    d, m = r.randint(1, 28), r.randint(1, 12)
    y = r.choice((2023, 2024, 2025))
    hh, mm = r.randint(0, 23), r.randint(0, 59)
    ys = f"{y}" if year4 else f"{y % 100:02d}"
    return f"{d:02d}.{m:02d}.{ys} {hh:02d}:{mm:02d}"


def _one(r: random.Random, v: Vocab) -> SynthSMS:
    ts = r.randint(1_690_000_000, 1_750_000_000)
    x = r.random()
    cur = r.choice(_CURRENCIES)
    card = f"{r.randint(0, 9999):04d}"
    if x < 0.55:
        merchant, city = _merchant(r, v), r.choice(v.cities)
        address = _address(r, v) if r.random() < 0.6 else ""
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
        merchant, city = _merchant(r, v), r.choice(v.cities)
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
    body = f"DECLINED: INSUFFICIENT FUNDS, {_merchant(r, v)}, card ***{card}"
    return SynthSMS(body, "funds", None, ts)


# traffic mixes (bench.py --traffic): "mixed" = every kind in its natural share (17 % are
# skipped by the parser's keyword filter and never reach the LLM); "purchase" = debit
# transactions only (the store-purchase and account-debit formats), every message
# LLM-routed -- the reference's BASELINE harness timed purchase bodies only
TRAFFIC_KINDS = {"mixed": None, "purchase": ("purchase", "account")}


def generate(n: int, seed: int = 0, unique: bool = True, vocab_name: str = "train",
             kinds: Optional[Sequence[str]] = None) -> List[SynthSMS]:
    """``n`` messages; with ``unique`` every body is distinct (defeats the response cache).
    ``vocab_name``: ``"train"`` (what the extractor is trained on) or ``"heldout"`` —
    merchant / city / street names disjoint from the training pools (held-out scoring
    and the benchmark's traffic).  ``kinds``: keep only these message kinds."""
    r = random.Random(seed)
    v = vocab(vocab_name)
    out: List[SynthSMS] = []
    seen = set()
    while len(out) < n:
        s = _one(r, v)
        if kinds is not None and s.kind not in kinds:
            continue
        if unique:
            if s.body in seen:
                continue
            seen.add(s.body)
        out.append(s)
    return out


def generate_bodies(n: int, seed: int = 0, vocab_name: str = "train") -> List[str]:
    return [s.body for s in generate(n, seed, vocab_name=vocab_name)]


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
    """Tokenizer-training text: bodies, normalised bodies and answer values
    (``"tokenizer"`` vocabulary: real training-split words only)."""
    from ..parse.text import normalize_body

    for s in generate(n, seed, unique=False, vocab_name="tokenizer"):
        yield s.body
        yield normalize_body(s.body)
        if s.answer:
            yield " ".join(v for v in s.answer.values() if v)
