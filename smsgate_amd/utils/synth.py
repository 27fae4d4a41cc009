"""Synthetic bank-notification SMS with ground-truth fields.

There is no dataset on the box (and the reference ships none — its only
fixtures are the three CASES of tests/test_parsers.py:11-58), so every
benchmark and tokenizer corpus here is generated.

Two generators share one output type (:class:`SynthSMS`):

* the **legacy mix** (``generate(..., families=None)``): the reference's two
  real-world purchase formats — ``APPROVED PURCHASE DB SALE: MERCHANT, CITY[,
  ADDRESS],dd.mm.yy HH:MM,card ***NNNN. Amount:X CUR, Balance:Y CUR``
  (process_cached.py:98-120) and the multi-line ``DEBIT ACCOUNT&#10;…`` format of
  test case 3 — plus credit / OTP / insufficient-funds notifications
  (worker-skipped kinds);
* **template families** (``families="train" | "heldout" | "all" | [names]``):
  :data:`FAMILIES` — 24 hand-written bank-SMS layouts plus 5 procedural ones
  (a random layout per message, training only) in English, Russian (Cyrillic) and
  Russian transliterated to Latin: different field orders and separators, label
  words (``Amount`` / ``Amt`` / ``Сумма`` / ``Summa``…), date styles
  (``dd.mm.yy HH:MM``, ``yyyy-mm-dd``, ``dd/mm/yyyy``, ``10 Jun 2025``, time
  first…), currency as a code or a symbol before / after the number (``$``,
  ``€``, ``֏``, ``₽``, ``руб.``), card masks (``*1234``, ``****1234``,
  ``4083***7538``, ``ending 1234``…), single- vs multi-line, optional address /
  balance, debit and credit.  The split is **by family**: :data:`HELDOUT_FAMILIES`
  never occur in training, so scoring on them measures what the Gemini prompt
  (gemini_parser.py:37-43, a format-agnostic instruction) is for — formats the
  extractor has never seen.  The legacy formats are train families.

Each item carries the body, the LLM answer (the nine strings the extractor
copies from the body, the Gemini JSON shape) and ``expected`` — the final
normalised values (``datetime``, ``Decimal``, ISO currency, 4-digit card) a
correct parse must produce, computed by the generator itself rather than by the
pipeline under test.  :func:`generate` is deterministic for a seed.
"""
from __future__ import annotations

import os
import random
import zlib
from dataclasses import dataclass, field
from datetime import datetime
from decimal import Decimal
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Tuple, Union

__all__ = ["SynthSMS", "generate", "generate_bodies", "generate_traffic", "reference_cases", "vocab", "Vocab",
           "TRAFFIC_KINDS", "TRAFFIC", "FAMILIES", "TRAIN_FAMILIES", "HELDOUT_FAMILIES", "family_names",
           "NEG_FAMILIES", "NEG_TRAIN_FAMILIES", "NEG_HELDOUT_FAMILIES", "VALUE_FAMILIES", "VALUE_HELDOUT_FAMILIES",
           "HELDOUT_VALUE_STYLES", "is_negative", "rejection_answer", "NEGATIVE_TXN"]

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
# the worker's skip keywords (parse/text.py) must not occur as whole words in a generated
# transaction: "OTP" / "CODE" / "PASS" as a merchant name would be skipped before the LLM
_SKIP_WORDS = frozenset({"OTP", "CODE", "PASS"})


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
    seen = set(_GOLDEN_VOCAB) | _SKIP_WORDS
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


# Latin -> Cyrillic letter map for Russian-language families (digraphs first): pseudo
# names keep their syllable structure, so Cyrillic merchants are as unpredictable as Latin
_CYR_DI = (("KH", "Х"), ("SH", "Ш"), ("TS", "Ц"), ("CH", "Ч"), ("YA", "Я"), ("OU", "У"), ("IO", "ИО"))
_CYR_1 = dict(zip("ABCDEFGHIJKLMNOPQRSTUVWXYZ", "АКЦДЕФГХИЖКЛМНОПКРСТУВВКЙЗ"))


def to_cyrillic(word: str) -> str:
    out, i = [], 0
    while i < len(word):
        for a, b in _CYR_DI:
            if word.startswith(a, i):
                out.append(b)
                i += len(a)
                break
        else:
            out.append(_CYR_1.get(word[i], word[i]))
            i += 1
    return "".join(out)


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
    family: str = "legacy"
    # final values of a correct parse (txn_type, date: datetime, amount / balance: Decimal,
    # currency: ISO code, card: 4 digits, merchant / city / address); None for skipped kinds
    expected: Optional[Dict[str, Any]] = field(default=None, repr=False)


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


def _dec(s: str) -> Decimal:
    from ..parse.numeric import parse_ambiguous_decimal

    return parse_ambiguous_decimal(s)


def _legacy_expected(ans: Dict[str, str]) -> Dict[str, Any]:
    return dict(txn_type=ans["txn_type"], date=datetime.strptime(ans["date"], "%d.%m.%Y %H:%M")
                if len(ans["date"]) == 16 else datetime.strptime(ans["date"], "%d.%m.%y %H:%M"),
                amount=_dec(ans["amount"]), currency=ans["currency"], card=ans["card"].replace("*", "")[-4:],
                merchant=ans["merchant"], city=ans["city"], address=ans["address"], balance=_dec(ans["balance"]))


def _legacy_purchase(r: random.Random, v: Vocab, ts: int, cur: str, card: str) -> SynthSMS:
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
    return SynthSMS(body, "purchase", ans, ts, "legacy_purchase", _legacy_expected(ans))


def _legacy_account(r: random.Random, v: Vocab, ts: int, cur: str, card: str) -> SynthSMS:
    merchant, city = _merchant(r, v), r.choice(v.cities)
    date = _date(r, year4=True)
    amt, bal = _amount(r, cur), _amount(r, cur)
    first = f"{r.randint(1000, 9999)}"
    body = (f"DEBIT ACCOUNT&#10;{amt} {cur}&#10;{first}***{card},&#10;{merchant}, {city}"
            f"&#10;{date}&#10;BALANCE: {bal} {cur}")
    ans = dict(txn_type="debit", date=date, amount=amt, currency=cur, card=card, merchant=merchant,
               city=city, address="", balance=bal)
    return SynthSMS(body, "account", ans, ts, "legacy_account", _legacy_expected(ans))


def _legacy_credit(r: random.Random, ts: int, cur: str, card: str,
                   kinds: Optional[Tuple[str, ...]] = None) -> SynthSMS:
    kind = r.choice(kinds or ("CREDIT PAYMENT", "C2C RECEIVED", "TRANSFER IN"))
    date = _date(r)
    amt, bal = _amount(r, cur), _amount(r, cur)
    body = f"{kind}: {date},card ***{card}. Amount:{amt} {cur}, Balance:{bal} {cur}"
    ans = dict(txn_type="credit", date=date, amount=amt, currency=cur, card=f"***{card}", merchant="",
               city="", address="", balance=bal)
    return SynthSMS(body, "credit", ans, ts, "legacy_credit", _legacy_expected(ans))


def _one(r: random.Random, v: Vocab) -> SynthSMS:
    ts = r.randint(1_690_000_000, 1_750_000_000)
    x = r.random()
    cur = r.choice(_CURRENCIES)
    card = f"{r.randint(0, 9999):04d}"
    if x < 0.55:
        return _legacy_purchase(r, v, ts, cur, card)
    if x < 0.80:
        return _legacy_account(r, v, ts, cur, card)
    if x < 0.90:
        return _legacy_credit(r, ts, cur, card)
    if x < 0.96:
        code = r.randint(100000, 999999)
        body = r.choice((f"Your OTP code: {code}. Do not share it.", f"CODE: {code} for login",
                         f"PASS={code} valid 5 min"))
        return SynthSMS(body, "otp", None, ts, "legacy_otp")
    body = f"DECLINED: INSUFFICIENT FUNDS, {_merchant(r, v)}, card ***{card}"
    return SynthSMS(body, "funds", None, ts, "legacy_funds")


# ---------------------------------------------------------------- template families
# currency symbols / words and the ISO code a correct parse maps them to
# (parse/canonical.py CURRENCY_ALIASES is the parse-side table; tests pin they agree)
_SYMBOL = {"USD": "$", "EUR": "€", "AMD": "֏", "RUB": "₽", "GEL": "₾", "GBP": "£"}
_WORD = {"RUB": "руб.", "AMD": "драм"}
_FAMILY_CURRENCIES = ("AMD", "USD", "EUR", "RUB", "GEL", "GBP")

# date styles: strftime format, whether the time of day is part of the value
_DATE_STYLES: Dict[str, Tuple[str, bool]] = {
    "dmy2": ("%d.%m.%y %H:%M", True),
    "dmy4": ("%d.%m.%Y %H:%M", True),
    "dmy4_date": ("%d.%m.%Y", False),
    "dmy2_date": ("%d.%m.%y", False),
    "iso": ("%Y-%m-%d %H:%M", True),
    "iso_t": ("%Y-%m-%dT%H:%M:%S", True),
    "slash": ("%d/%m/%Y %H:%M", True),
    "mon": ("%d %b %Y %H:%M", True),
    "mon_up": ("%d-%b-%Y %H:%M", True),
    "time_first": ("%H:%M %d.%m.%Y", True),
    # the value grammar's other axes (VERDICT r05 next #1a): month-first order, full
    # month names, 12-hour clocks (zero-padded or not, glued or spaced, upper or lower
    # case, time after or before the date), Russian month names in every combination but
    # the held-out one.  Each held-out style below is a combination of axes that all occur
    # here, never the combination itself (tests/test_families.py pins both)
    "mdy_mon": ("%b %d, %Y %H:%M", True),  # "Jun 06, 2025 14:23"
    "mdy_mon_date": ("%b %-d, %Y", False),  # "Jun 6, 2025"
    "full_month": ("%-d %B %Y %H:%M", True),  # "6 June 2025 14:23"
    "dmy4_12h": ("%d.%m.%Y %I:%M %p", True),  # "06.06.2025 02:23 PM"
    "slash_12h": ("%d/%m/%Y %-I:%M%p", True),  # "06/06/2025 2:23PM"
    "mon_12h": ("%-d %b %Y %-I:%M %p", True),  # "6 Jun 2025 2:23 PM"
    "iso_12h": ("%Y-%m-%d %I:%M %p", True),  # "2025-06-06 02:23 pm" (lower case)
    "time_first_12h": ("%-I:%M %p %d.%m.%Y", True),  # "2:23 PM 06.06.2025"
    "ru_month_date": ("", False),  # "6 июня 2025"
    "ru_month_g": ("", True),  # "6 июня 2025 г. 14:23"
    "ru_month_v": ("", True),  # "6 июня 2025 в 14:23"
    "ru_time_month": ("", True),  # "14:23 6 июня 2025"
    "ru_mon_abbr": ("", True),  # "6 июн. 2025 14:23" / "06 июн 2025 14:23"
    "tr_month": ("", True),  # "6 iyunya 2025 14:23" (transliterated genitive)
    # held-out VALUE styles (never in a training pool: only the heldout_values families
    # below render them; tests/test_families.py pins it)
    "en_12h": ("%b %-d, %Y %-I:%M %p", True),  # "Jun 6, 2025 2:23 PM"
    "ru_month": ("", True),  # "6 июня 2025 14:23" (Russian month name, genitive)
}
_RU_MONTHS_GEN = ("января", "февраля", "марта", "апреля", "мая", "июня", "июля", "августа", "сентября",
                  "октября", "ноября", "декабря")
# short forms: "май" (not the genitive "мая", which would be the held-out style itself)
_RU_MONTHS_ABBR = ("янв", "фев", "мар", "апр", "май", "июн", "июл", "авг", "сен", "окт", "ноя", "дек")
_TR_MONTHS_GEN = ("yanvarya", "fevralya", "marta", "aprelya", "maya", "iyunya", "iyulya", "avgusta", "sentyabrya",
                  "oktyabrya", "noyabrya", "dekabrya")
# held-out value styles of every kind (dates above, money / number / card styles below)
HELDOUT_VALUE_STYLES = {"dates": ("en_12h", "ru_month"), "money": ("code_glued",), "numbers": ("apos",),
                        "cards": ("x_mask", "dots_mask")}
# per language: date styles, money layouts, number formats, card masks
_STYLE_POOLS = {
    "en": dict(dates=("dmy2", "dmy4", "iso", "iso_t", "slash", "mon", "mon_up", "mdy_mon", "mdy_mon_date",
                      "full_month", "dmy4_12h", "slash_12h", "mon_12h", "iso_12h", "time_first_12h"),
               money=("code_after", "code_after", "code_before", "sym_before", "sym_after"),
               numbers=("dot", "comma_dot", "comma_dot", "int"),
               cards=("star1", "stars2", "stars3", "stars4", "spaced", "first_mask", "ending", "xx_mask", "dots3",
                      "x_groups")),
    "ru": dict(dates=("dmy2", "dmy4", "dmy4_date", "dmy2_date", "time_first", "iso", "ru_month_date", "ru_month_g",
                      "ru_month_v", "ru_time_month", "ru_mon_abbr"),
               money=("code_after", "code_after", "code_before", "sym_after", "word_after"),
               numbers=("space_comma", "space_comma", "comma", "dot", "int"),
               cards=("star1", "stars2", "stars4", "spaced", "first_mask", "xx_mask", "dots3")),
    "tr": dict(dates=("dmy2", "dmy4", "time_first", "iso", "slash", "tr_month", "tr_month"),
               money=("code_after", "code_before", "sym_after"),
               numbers=("dot", "comma", "space_comma", "comma_dot"),
               cards=("star1", "stars2", "stars4", "first_mask", "xx_mask", "dots3", "x_groups")),
}
_NOISE = {
    "en": ("", "", "", " Thank you.", " Details in the app.", " Bank."),
    "ru": ("", "", "", " Спасибо!", " Подробнее в приложении."),
    "tr": ("", "", "", " Spasibo!", " Podrobnee v prilozhenii."),
}


def _fmt_number(r: random.Random, style: str, v: Decimal, cur: str) -> str:
    if style == "int" and cur not in ("AMD", "RUB"):
        style = "dot"
    if style == "int":
        return str(int(v))
    q = f"{v:.2f}"
    whole, frac = q.split(".")
    if style == "dot":
        return q
    if style == "comma":
        return f"{whole},{frac}"
    grouped = f"{int(whole):,}"
    if style == "comma_dot":
        return f"{grouped}.{frac}"
    if style == "space_comma":
        return f"{grouped.replace(',', ' ')},{frac}"
    if style == "apos":  # held-out value style: apostrophe thousands ("1'234.56")
        return f"{grouped.replace(',', chr(39))}.{frac}"
    raise ValueError(style)


class _Ctx:
    """Values of one message, rendered in the family's styles; every value a
    template writes is recorded as the answer (the exact body substring)."""

    def __init__(self, r: random.Random, v: Vocab, fam: "Family", ts: int) -> None:
        self.r, self.v, self.fam, self.ts = r, v, fam, ts
        pools = _STYLE_POOLS[fam.lang]
        self.cur = r.choice(fam.currencies or _FAMILY_CURRENCIES)
        self.money = r.choice(fam.money or pools["money"])
        if self.money.startswith("sym") and self.cur not in _SYMBOL:
            self.money = "code_after"
        if self.money == "word_after" and self.cur not in _WORD:
            self.money = "code_after"
        self.num_style = r.choice(fam.numbers or pools["numbers"])
        self.date_style = r.choice(fam.dates or pools["dates"])
        self.card_style = r.choice(fam.cards or pools["cards"])
        noise = _label_noise() if fam.name.startswith("proc_") else 0.0
        if noise > 0 and r.random() < noise * 0.5:  # (off: no draw, the default stream is unchanged)
            # a "#1234" mask: one more mask shape than the fixed families use, so an unseen
            # one reads as a card, not as merchant text ("№1234" is no valid span: the
            # tokenizer glues the sign's bytes to the first digit)
            self.card_style = "hash"
        cyr = fam.lang == "ru" and r.random() < 0.5
        self.cyr = cyr
        self.case = r.choice(fam.cases)
        self.ans: Dict[str, str] = dict(txn_type=fam.txn, date="", amount="", currency="", card="", merchant="",
                                        city="", address="", balance="")
        self.exp: Dict[str, Any] = dict(txn_type=fam.txn, amount=Decimal("0.0"), currency=None, card=None,
                                        merchant="", city="", address="", balance=Decimal("0.0"))

    # ---- names
    def _name(self, w: str) -> str:
        if self.cyr:
            w = to_cyrillic(w)
        return w.title() if self.case == "title" else w

    def M(self) -> str:
        m = " ".join(self._name(self.r.choice(self.v.words)) for _ in range(self.r.choice((1, 1, 2, 2, 3))))
        if self.r.random() < 0.06:
            m += f" {self.r.randint(1, 999)}"
        self.ans["merchant"] = self.exp["merchant"] = m
        return m

    def C(self) -> str:
        c = self._name(self.r.choice(self.v.cities))
        self.ans["city"] = self.exp["city"] = c
        return c

    def A(self) -> str:
        st = self._name(self.r.choice(self.v.streets))
        n = self.r.randint(1, 150)
        if self.fam.lang == "ru":
            a = f"{self.r.choice(('ул.', 'пр.', 'ул.'))} {st} {n}"
        elif self.fam.lang == "tr":
            a = f"{self.r.choice(('ul.', 'pr.'))} {st} {n}"
        else:
            sfx = self.r.choice(_STREET_SUFFIXES)
            a = f"{st} {sfx.title() if self.case == 'title' else sfx} {n}"
        self.ans["address"] = self.exp["address"] = a
        return a

    # ---- date
    def D(self) -> str:
        r = self.r
        fmt, timed = _DATE_STYLES[self.date_style]
        dt = datetime(r.choice((2023, 2024, 2025)), r.randint(1, 12), r.randint(1, 28),
                      r.randint(0, 23), r.randint(0, 59), r.randint(0, 59) if "%S" in fmt else 0)
        if not timed:
            dt = dt.replace(hour=0, minute=0, second=0)
        st = self.date_style
        hm = f"{dt.hour:02d}:{dt.minute:02d}"
        if st == "ru_month":
            s = f"{dt.day} {_RU_MONTHS_GEN[dt.month - 1]} {dt.year} {hm}"
        elif st.startswith("ru_"):
            dm = f"{dt.day} {_RU_MONTHS_GEN[dt.month - 1]} {dt.year}"
            if st == "ru_month_date":
                s = dm
            elif st == "ru_month_g":
                s = f"{dm} г. {hm}"
            elif st == "ru_month_v":
                s = f"{dm} в {hm}"
            elif st == "ru_time_month":
                s = f"{hm} {dm}"
            else:  # ru_mon_abbr
                d = f"{dt.day:02d}" if r.random() < 0.5 else f"{dt.day}"
                s = f"{d} {_RU_MONTHS_ABBR[dt.month - 1]}{r.choice(('.', ''))} {dt.year} {hm}"
        elif st == "tr_month":
            s = f"{dt.day} {_TR_MONTHS_GEN[dt.month - 1]} {dt.year} {hm}"
        else:
            s = dt.strftime(fmt)
        if st == "mon_up":
            s = s.upper()
        elif st == "iso_12h":
            s = s.lower()
        self.ans["date"] = s
        self.exp["date"] = dt
        return s

    # ---- money
    def _value(self) -> Decimal:
        big = self.cur in ("AMD", "RUB")
        v = self.r.uniform(100, 250000) if big else self.r.uniform(1, 5000)
        return Decimal(f"{v:.2f}")

    def _money(self, key: str) -> str:
        v = self._value()
        num = _fmt_number(self.r, self.num_style, v, self.cur)
        if self.num_style == "int" and self.cur in ("AMD", "RUB"):
            v = Decimal(int(v))
        cur = {"code_after": self.cur, "code_before": self.cur, "sym_before": _SYMBOL.get(self.cur),
               "sym_after": _SYMBOL.get(self.cur), "word_after": _WORD.get(self.cur),
               "code_glued": self.cur}[self.money]
        cur_value = cur[:-1] if cur.endswith(".") else cur  # "руб." -> the word, not its dot
        if self.money == "code_before":
            s = f"{cur} {num}"
        elif self.money == "code_glued":  # held-out value style: "USD52.00"
            s = f"{cur}{num}"
        elif self.money == "sym_before":
            s = f"{cur}{num}"
        elif self.money == "sym_after" and self.r.random() < 0.3:
            s = f"{num}{cur}"
        else:
            s = f"{num} {cur}"
        self.ans[key] = num
        self.exp[key] = v
        if not self.ans["currency"]:
            self.ans["currency"] = cur_value
            self.exp["currency"] = self.cur
        return s

    def AMT(self) -> str:
        return self._money("amount")

    def BAL(self) -> str:
        return self._money("balance")

    # ---- card
    def CARD(self) -> str:
        c = f"{self.r.randint(0, 9999):04d}"
        st = self.card_style
        if st == "first_mask":  # normalize_body masks it to CARD:NNNN (gemini_parser.py:121-137)
            s, a = f"{self.r.randint(1000, 9999)}***{c}", c
        elif st == "spaced":
            s, a = f"**** {c}", c
        elif st == "ending":
            s, a = f"ending {c}", c
        elif st == "hash":
            s, a = f"#{c}", c
        elif st == "xx_mask":  # "XX1234", "xxxx1234", "XXXX 1234" (one glyph: the held-out x_mask)
            s, a = f"{self.r.choice('xX') * self.r.randint(2, 4)}{self.r.choice(('', '', ' '))}{c}", c
        elif st == "dots3":  # "...1234", "…1234" (two dots: the held-out dots_mask)
            s, a = f"{self.r.choice(('...', '…'))}{c}", c
        elif st == "x_groups":  # "XXXX XXXX XXXX 1234"
            s, a = f"{' '.join([self.r.choice(('XXXX', 'xxxx', '****'))] * 3)} {c}", c
        elif st == "x_mask":  # held-out value style
            s, a = f"x{c}", c
        elif st == "dots_mask":  # held-out value style
            s, a = f"..{c}", c
        else:
            stars = {"star1": "*", "stars2": "**", "stars3": "***", "stars4": "****"}[st]
            s = a = f"{stars}{c}"
        self.ans["card"] = a
        self.exp["card"] = c
        return s

    def pick(self, *opts: str) -> str:
        return self.r.choice(opts)

    def noise(self) -> str:
        return self.r.choice(_NOISE[self.fam.lang])


@dataclass(frozen=True)
class Family:
    name: str
    lang: str  # en | ru | tr (Russian in Latin letters)
    txn: str  # debit | credit
    render: Callable[[_Ctx], str]
    heldout: bool = False
    cases: Tuple[str, ...] = ("upper",)
    dates: Tuple[str, ...] = ()  # () = the language's pool
    money: Tuple[str, ...] = ()
    cards: Tuple[str, ...] = ()
    currencies: Tuple[str, ...] = ()
    numbers: Tuple[str, ...] = ()
    # "formats" (a new layout, the default), "values" (a training layout rendered in
    # held-out value styles) or "negative" (not a transaction: txn "unknown" / "otp")
    split: str = "formats"


def _opt(c: _Ctx, p: float, f: Callable[[], str], pre: str = ", ") -> str:
    return pre + f() if c.r.random() < p else ""


# Labels are shared across families (each family draws from the language's synonyms),
# so a held-out family is a NEW LAYOUT of label words the model has seen elsewhere.
def _bal_en(c: _Ctx) -> str:
    return c.pick("Balance", "Bal", "Avail. balance", "Available", "Avl bal", "Remaining balance")


def _bal_ru(c: _Ctx) -> str:
    return c.pick("Остаток", "Баланс", "Доступно")


def _bal_tr(c: _Ctx) -> str:
    return c.pick("ostatok", "Ostatok", "dostupno", "Dostupno", "balans")


FAMILIES: Tuple[Family, ...] = (
    # ---- English, training
    Family("en_card_at", "en", "debit", lambda c: (
        f"{c.pick('Card', 'CARD', 'card')} {c.CARD()}: {c.pick('purchase', 'Purchase', 'POS purchase', 'payment')} "
        f"{c.AMT()} at {c.M()}, {c.C()}{_opt(c, 0.3, c.A)}. {c.D()}. {_bal_en(c)} {c.BAL()}{c.noise()}"),
        cases=("upper", "upper", "title")),
    Family("en_pipe", "en", "debit", lambda c: (
        f"{c.M()} | {c.C()} | {c.AMT()} | card {c.CARD()} | {c.D()} | {_bal_en(c)} {c.BAL()}")),
    Family("en_ml_labels", "en", "debit", lambda c: (
        f"{c.pick('Purchase', 'PURCHASE', 'Payment', 'Card payment')}\n{c.pick('Card', 'Card no')}: {c.CARD()}\n"
        f"{c.pick('Amount', 'Amt', 'Sum')}: {c.AMT()}\n{c.pick('Merchant', 'Shop', 'Payee')}: {c.M()}\n"
        f"{c.pick('City', 'Location')}: {c.C()}\n{c.pick('Date', 'Time')}: {c.D()}\n{_bal_en(c)}: {c.BAL()}"),
        cases=("upper", "title")),
    Family("en_you_paid", "en", "debit", lambda c: (
        f"You {c.pick('paid', 'spent')} {c.AMT()} {c.pick('to', 'at')} {c.M()} in {c.C()} with card {c.CARD()} "
        f"on {c.D()}. {_bal_en(c)} {c.BAL()}{c.noise()}"), cases=("title", "upper")),
    Family("en_pos_semicolon", "en", "debit", lambda c: (
        f"{c.pick('POS PURCHASE', 'POS', 'PURCHASE')} {c.AMT()}; {c.M()}; {c.A()}, {c.C()}; card {c.CARD()}; "
        f"{c.D()}; bal: {c.BAL()}")),
    Family("en_charged_nobal", "en", "debit", lambda c: (
        f"{c.pick('Card', 'Your card')} {c.CARD()} was charged {c.AMT()} at {c.M()}, {c.C()} on {c.D()}.{c.noise()}"),
        cases=("upper", "title")),
    Family("en_upper_compact", "en", "debit", lambda c: (
        f"DEBIT {c.AMT()} CARD{c.CARD()} {c.M()}/{c.C()} {c.D()} BAL:{c.BAL()}"),
        cards=("star1", "stars2", "stars3", "stars4")),
    Family("en_internet", "en", "debit", lambda c: (
        f"{c.pick('Internet purchase', 'Online payment', 'E-commerce purchase')} {c.AMT()} {c.M()} card {c.CARD()} "
        f"{c.D()}. {_bal_en(c)}: {c.BAL()}")),
    Family("en_location_ml", "en", "debit", lambda c: (
        f"TRANSACTION: {c.pick('PURCHASE', 'POS', 'PAYMENT')}\nAMOUNT: {c.AMT()}\nCARD: {c.CARD()}\n"
        f"MERCHANT: {c.M()}\nLOCATION: {c.C()}, {c.A()}\nDATE: {c.D()}\nBALANCE: {c.BAL()}")),
    Family("en_bracket", "en", "debit", lambda c: (
        f"[{c.M()}] [{c.C()}] {c.AMT()} card {c.CARD()} {c.D()} {c.pick('balance', 'bal')} {c.BAL()}")),
    Family("en_refund", "en", "credit", lambda c: (
        f"{c.pick('Refund', 'Reversal', 'Credit')} {c.AMT()} to card {c.CARD()} from {c.M()}, {c.C()} on {c.D()}. "
        f"{_bal_en(c)} {c.BAL()}")),
    # ---- Russian (Cyrillic), training
    Family("ru_pokupka", "ru", "debit", lambda c: (
        f"{c.pick('Покупка', 'Оплата', 'Списание')} {c.AMT()} {c.M()}, {c.C()}{_opt(c, 0.3, c.A)}. "
        f"{c.pick('Карта', 'карта')} {c.CARD()}. {c.D()}. {_bal_ru(c)} {c.BAL()}{c.noise()}")),
    Family("ru_oplata_ml", "ru", "debit", lambda c: (
        f"{c.pick('Оплата', 'Покупка')}\n{c.pick('Карта', 'карта')} {c.CARD()}\n{c.pick('Сумма', 'Списано')}: "
        f"{c.AMT()}\n{c.M()}\n{c.C()}\n{c.D()}\n{_bal_ru(c)}: {c.BAL()}")),
    Family("ru_spisanie", "ru", "debit", lambda c: (
        f"{c.D()} {c.pick('Списание', 'Покупка')} {c.AMT()}, карта {c.CARD()}, {c.M()}, г. {c.C()}. "
        f"{_bal_ru(c)}: {c.BAL()}")),
    Family("ru_nobal", "ru", "debit", lambda c: (
        f"Покупка по карте {c.CARD()} на {c.AMT()}{c.pick(': ', ' в ')}{c.M()}, {c.C()}. {c.D()}{c.noise()}")),
    Family("ru_zachislenie", "ru", "credit", lambda c: (
        f"{c.pick('Зачисление', 'Возврат')} {c.AMT()} на карту {c.CARD()} от {c.M()}. {c.D()}. "
        f"{_bal_ru(c)}: {c.BAL()}")),
    # ---- Russian transliterated, training
    Family("tr_pokupka_ml", "tr", "debit", lambda c: (
        f"{c.pick('Pokupka', 'Oplata')}: {c.AMT()}\n{c.pick('Karta', 'karta')}: {c.CARD()}\n"
        f"{c.pick('Mesto', 'Magazin')}: {c.M()}, {c.C()}\n{c.pick('Data', 'Vremya')}: {c.D()}\n"
        f"{_bal_tr(c).title()}: {c.BAL()}")),
    Family("tr_spisanie", "tr", "debit", lambda c: (
        f"{c.pick('Spisanie', 'Pokupka', 'Summa')} {c.AMT()} s karty {c.CARD()}. {c.M()}, {c.C()}. {c.D()}. "
        f"{_bal_tr(c).title()}: {c.BAL()}{c.noise()}")),
    # ---- held out: new layouts of seen label words (never trained on)
    Family("en_alert", "en", "debit", lambda c: (
        f"Debit alert: {c.AMT()} spent on card {c.CARD()} at {c.M()}, {c.C()} on {c.D()}. "
        f"{_bal_en(c)}: {c.BAL()}"), heldout=True, cases=("upper", "title")),
    Family("en_amount_first", "en", "debit", lambda c: (
        f"{c.AMT()} debited from card {c.CARD()} at {c.M()}, {c.C()}, {c.A()} on {c.D()}. "
        f"{_bal_en(c)} {c.BAL()}.{c.noise()}"), heldout=True),
    Family("en_reverse_pipe", "en", "debit", lambda c: (
        f"{_bal_en(c)} {c.BAL()} | {c.D()} | -{c.AMT()} | {c.M()}, {c.C()} | {c.CARD()}"), heldout=True,
        cards=("star1", "stars2", "stars3", "stars4")),
    Family("ru_karta_first", "ru", "debit", lambda c: (
        f"Карта {c.CARD()} {c.D()} покупка на сумму {c.AMT()} в {c.M()}, {c.C()}, {c.A()}. "
        f"{_bal_ru(c)} {c.BAL()}"), heldout=True),
    Family("ru_ml_addr", "ru", "debit", lambda c: (
        f"Карта {c.CARD()}\nПокупка {c.AMT()}\n{c.M()}\n{c.A()}\n{c.C()}\n{_bal_ru(c)} {c.BAL()}\n{c.D()}"),
        heldout=True),
    Family("tr_oplata", "tr", "debit", lambda c: (
        f"Oplata {c.AMT()} {c.M()}, {c.C()}; karta {c.CARD()}; {c.D()}; {_bal_tr(c)} {c.BAL()}"), heldout=True),
)
# ---------------------------------------------------------------- procedural layouts
# Training-only families whose layout is drawn per message: the five segments (amount,
# card, place = merchant / city / address, date, balance) in a random order, an optional
# header word, random separators or one segment per line, each segment labelled or not
# (label words from the language's pools), place rendered in one of several shapes,
# optional address / balance.  They teach field SEMANTICS rather than template
# positions.  The (language, segment order, multi-line) signatures of the held-out
# families are excluded (_HELDOUT_SIGNATURES, pinned by tests/test_families.py), and
# the held-out families' own phrasings ("Debit alert", "spent on card", "debited from",
# "покупка на сумму") are not in the pools: a held-out layout stays unseen.
_PROC_POOLS = {
    "en": dict(
        head_debit=("Purchase", "PURCHASE", "POS", "Payment", "Card payment", "DEBIT", "Debit", "Charge", "POS PURCHASE"),
        head_credit=("Refund", "Credit", "Reversal", "Incoming transfer", "REFUND", "Payment received",
                     "Credited", "Deposit", "Transfer received", "Money received"),
        amt=("Amount", "Amt", "Sum", "Total", "AMOUNT"), card=("card", "Card", "CARD", "Card no"),
        merch=("Merchant", "Shop", "Payee", "MERCHANT"), city=("City", "Location", "CITY"),
        merch_credit=("From", "Sender", "Payer", "Remitter"), credited=("credited", "received", "deposited"),
        to_card=("to card", "to your card", "to account"),
        addr=("Address", "Addr"), date=("Date", "Time", "DATE"),
        bal=("Balance", "Bal", "Avail. balance", "Available", "Avl bal", "Remaining balance", "BALANCE", "Bal."),
        at=("at", "AT"), on=("on",), inn=("in",)),
    "ru": dict(
        head_debit=("Покупка", "Оплата", "Списание", "ПОКУПКА", "Оплата товаров"),
        head_credit=("Зачисление", "Возврат", "Пополнение", "Поступление", "Перевод получен"),
        amt=("Сумма", "Списано", "Сумма операции"), card=("Карта", "карта", "по карте", "КАРТА"),
        merch=("Магазин", "Место", "Получатель"), city=("Город",), addr=("Адрес",), date=("Дата", "Время"),
        merch_credit=("Отправитель", "От"), credited=("зачислено", "поступило"), to_card=("на карту", "на счет"),
        bal=("Остаток", "Баланс", "Доступно", "Доступный остаток"),
        at=("в",), on=("",), inn=("г.",)),
    "tr": dict(
        head_debit=("Pokupka", "Oplata", "Spisanie", "POKUPKA"),
        head_credit=("Zachislenie", "Vozvrat", "Popolnenie", "Postuplenie"),
        amt=("Summa", "Spisano"), card=("karta", "Karta", "po karte", "s karty"),
        merch=("Mesto", "Magazin", "Poluchatel"), city=("Gorod",), addr=("Adres",), date=("Data", "Vremya"),
        merch_credit=("Otpravitel", "Ot"), credited=("zachisleno", "postupilo"), to_card=("na kartu", "na schet"),
        bal=("ostatok", "Ostatok", "dostupno", "Dostupno", "balans", "Balans"),
        at=("v",), on=("",), inn=("g.",)),
}
_SEGMENTS = ("AMT", "CARD", "PLACE", "DATE", "BAL")
# (language, segment order, one segment per line) of every held-out family: never drawn
_HELDOUT_SIGNATURES = frozenset({
    ("en", ("AMT", "CARD", "PLACE", "DATE", "BAL"), False),  # en_alert, en_amount_first
    ("en", ("BAL", "DATE", "AMT", "PLACE", "CARD"), False),  # en_reverse_pipe
    ("ru", ("CARD", "DATE", "AMT", "PLACE", "BAL"), False),  # ru_karta_first
    ("ru", ("CARD", "AMT", "PLACE", "BAL", "DATE"), True),  # ru_ml_addr
    ("tr", ("AMT", "PLACE", "CARD", "DATE", "BAL"), False),  # tr_oplata
})


def _label_noise() -> float:
    """Share of procedural labels drawn as an unseen pseudo-word ("Vokta: ..."), so that
    the extractor learns that any "Word:" before a value is a label, not part of it (a
    held-out "Sender: NAME" otherwise leaks into the merchant).  SMSGATE_SYNTH_LABELS
    overrides it for training-mix experiments (scripts/qa_probe.py --variants)."""
    return float(os.environ.get("SMSGATE_SYNTH_LABELS", _LABEL_NOISE))


_LABEL_NOISE = 0.0


def _proc_layout(r: random.Random, lang: str) -> Tuple[Tuple[str, ...], bool]:
    while True:
        order = list(_SEGMENTS)
        r.shuffle(order)
        if r.random() < 0.25:
            order.remove("BAL")
        multi = r.random() < 0.3
        if (lang, tuple(order), multi) not in _HELDOUT_SIGNATURES:
            return tuple(order), multi


_FILLER_LETTERS = {"en": "abcdefghiklmnoprstuvwy", "tr": "abdeghiklmnoprstuvyz",
                   "ru": "абвгдеийклмнопрстуфхчшыя"}


def _filler(r: random.Random, lang: str) -> str:
    """One or two pseudo-words: a connector phrase the extractor has never seen
    ("na summu", "spent on card" in a new layout).  Inserted before values so that the
    model learns to read an unknown phrase as filler, not as a field."""
    a = _FILLER_LETTERS[lang]
    return " ".join("".join(r.choice(a) for _ in range(r.randint(2, 6))) for _ in range(r.randint(1, 2)))


def _proc_render(c: "_Ctx") -> str:
    r, lang = c.r, c.fam.lang
    P = _PROC_POOLS[lang]
    order, multi = _proc_layout(r, lang)
    labelled = r.random() < 0.5  # "Label: value" style (else mostly bare values / prepositions)
    colon = r.choice((": ", ": ", " ", ":"))
    # this message carries up to two unknown connector phrases (bounded: random Cyrillic
    # letters cost a token each, and the body must stay inside the 128-token prompt)
    fills = [2 if r.random() < 0.4 else 0]

    def filler() -> str:
        fills[0] -= 1
        return _filler(r, lang)

    def want_fill(p: float) -> bool:
        return fills[0] > 0 and r.random() < p

    noise = _label_noise()

    def lab(pool: Sequence[str], unseen_ok: bool = True) -> str:
        # never for the balance: an amount and a balance are told apart by their label
        word = _filler(r, lang).split(" ")[0].title() if unseen_ok and noise and r.random() < noise \
            else r.choice(pool)
        return word + colon + (filler() + " " if want_fill(0.3) else "")

    segs: List[str] = []
    head = ""
    credit = c.fam.txn == "credit"
    # a credit is always announced (nothing else tells it from a debit); a debit's header
    # is optional -- an unlabelled transaction is a debit
    if c.fam.txn == "credit" or r.random() < 0.75:
        head = r.choice(P["head_credit"] if c.fam.txn == "credit" else P["head_debit"])
    for seg in order:
        if seg == "AMT":
            v = c.AMT()
            if credit and r.random() < 0.35:  # "2 500 RUB зачислено", "52.00 USD credited"
                v = v + " " + r.choice(P["credited"])
            elif r.random() < 0.15:  # a debit written as a negative amount ("-52.00 USD")
                v = "-" + v
            if labelled or r.random() < 0.2:
                v = lab(P["amt"]) + v
            elif want_fill(0.6):
                v = filler() + " " + v
            segs.append(v)
        elif seg == "CARD":
            v = c.CARD()
            if credit and r.random() < 0.3:  # "to card *1234", "на карту *1234"
                segs.append(r.choice(P["to_card"]) + " " + v)
            else:
                segs.append(lab(P["card"]) + v if (labelled or r.random() < 0.7) else v)
        elif seg == "DATE":
            v = c.D()
            if labelled and r.random() < 0.7:
                segs.append(lab(P["date"]) + v)
            elif lang == "en" and r.random() < 0.3:
                segs.append("on " + v)
            else:
                segs.append(v)
        elif seg == "BAL":
            v = c.BAL()
            segs.append(lab(P["bal"], False) + v)
        else:  # PLACE
            m = c.M()
            city = c.C() if r.random() < 0.85 else ""
            addr = c.A() if r.random() < 0.35 else ""
            if labelled and r.random() < 0.6:
                mlab = P["merch_credit"] if credit and r.random() < 0.6 else P["merch"]
                parts = [lab(mlab) + m] + ([lab(P["city"]) + city] if city else []) + \
                    ([lab(P["addr"]) + addr] if addr else [])
                segs.extend(parts) if multi else segs.append(", ".join(parts))
                continue
            shape = r.choice(("comma", "comma", "paren", "slash", "in", "lines"))
            # the merchant leads; city and address come in either order (an address is
            # recognised by its shape -- street word, number -- not by its position)
            addr_first = bool(addr) and r.random() < 0.4
            if not city:
                place = m + (", " + addr if addr else "")
            elif shape == "paren":
                place = f"{m} ({city})" + (f", {addr}" if addr else "")
            elif shape == "slash":
                place = f"{m}/{city}" + (f", {addr}" if addr else "")
            elif shape == "in":
                place = f"{m} {r.choice(P['inn'])} {city}" + (f", {addr}" if addr else "")
            elif shape == "lines" and multi:
                segs.extend([m] + ([addr, city] if addr_first else [city] + ([addr] if addr else [])))
                continue
            elif addr_first:
                place = f"{m}, {addr}, {city}"
            else:
                place = f"{m}, {city}" + (f", {addr}" if addr else "")
            if r.random() < 0.3:
                place = r.choice(P["at"]) + " " + place
            if want_fill(0.4):
                place = filler() + " " + place
            segs.append(place)
    if multi:
        body = "\n".join(([head] if head else []) + segs)
    else:
        seps = (", ", "; ", " | ", ". ", " ", " / ")
        sep = r.choice(seps)
        if r.random() < 0.25:  # mixed separators within one message
            body = segs[0] + "".join((sep if r.random() < 0.5 else r.choice(seps)) + x for x in segs[1:])
        else:
            body = sep.join(segs)
        if head and want_fill(0.4):
            head += " " + filler()
        body = (head + r.choice((": ", " ", ". ")) if head else "") + body
    return body + (c.noise() if not multi else "")


FAMILIES = FAMILIES + (
    Family("proc_en", "en", "debit", _proc_render, cases=("upper", "upper", "title")),
    Family("proc_en_credit", "en", "credit", _proc_render, cases=("upper", "title")),
    Family("proc_ru", "ru", "debit", _proc_render),
    Family("proc_ru_credit", "ru", "credit", _proc_render),
    Family("proc_tr", "tr", "debit", _proc_render),
)
_LAYOUT = {f.name: f.render for f in FAMILIES}

# ---------------------------------------------------------------- held-out VALUE styles
# a held-out layout is a new ordering / phrasing of value formats the
# model has seen; these families are TRAINING layouts rendered in value styles no training
# family ever emits (HELDOUT_VALUE_STYLES: 12-hour English and Russian month-name dates,
# a currency code glued to the number, apostrophe thousands, "x1234" / "..1234" card
# masks), plus one credit layout never trained on.  Scored as quality_heldout_values.
VALUE_FAMILIES: Tuple[Family, ...] = (
    Family("hv_en_12h", "en", "debit", _LAYOUT["en_card_at"], heldout=True, split="values", dates=("en_12h",),
           cases=("upper", "title")),
    Family("hv_ru_month", "ru", "debit", _LAYOUT["ru_pokupka"], heldout=True, split="values", dates=("ru_month",)),
    Family("hv_en_glued", "en", "debit", _LAYOUT["en_pipe"], heldout=True, split="values", money=("code_glued",)),
    Family("hv_en_apos", "en", "debit", _LAYOUT["en_ml_labels"], heldout=True, split="values", numbers=("apos",),
           cases=("upper", "title")),
    Family("hv_tr_cards", "tr", "debit", _LAYOUT["tr_spisanie"], heldout=True, split="values",
           cards=("x_mask", "dots_mask")),
    Family("hv_en_credit", "en", "credit", lambda c: (
        f"Incoming payment {c.AMT()} credited to card {c.CARD()}. Sender: {c.M()}, {c.C()}. {c.D()}. "
        f"{_bal_en(c)} {c.BAL()}"), heldout=True, split="values"),
)


# ---------------------------------------------------------------- non-transactions
# VERDICT r04 missing #1: Gemini classifies as well as extracts -- "txn_type может иметь
# значения 'debit', 'credit', 'otp' или 'unknown'" (gemini_parser.py:41); a
# non-transaction comes back with null fields, post-processing raises on str(None)
# (:235-241) and the worker dead-letters it as {"reason": "unmatched"}
# (worker.py:151-158).  These families are bank SMS that pass the worker's keyword
# filter but are NOT transactions: card blocked / unblocked, log-in alerts, cashback and
# promo offers carrying dates, amounts and merchant names, limit changes, balance-only
# statements, declines phrased without INSUFFICIENT FUNDS, P2P requests without a card,
# tariff notices, and confirmation numbers that avoid the OTP / CODE: keywords.  Their
# answer is txn_type "unknown" (or "otp") with every other field null.  Split by family
# like the formats: the held-out ones are a known concept in a new language / phrasing.
def _phone(c: _Ctx) -> str:
    r = c.r
    return r.choice((f"+374 10 {r.randint(100000, 999999)}", f"8-800-{r.randint(100, 999)}-{r.randint(10, 99)}-"
                     f"{r.randint(10, 99)}", f"*{r.randint(100, 9999)}", f"{r.randint(1000, 9999)}"))


def _digits(c: _Ctx) -> str:
    return f"{c.r.randint(0, 10 ** c.r.choice((4, 5, 6)) - 1):0{c.r.choice((4, 6))}d}"


def _pct(c: _Ctx) -> str:
    return str(c.r.choice((2, 3, 5, 7, 10, 15, 20, 25, 30, 50)))


NEG_FAMILIES: Tuple[Family, ...] = (
    # ---- training
    Family("neg_en_blocked", "en", "unknown", lambda c: c.pick(
        f"Your card {c.CARD()} has been blocked. To unblock it call {_phone(c)}.",
        f"Card {c.CARD()} is temporarily blocked due to suspicious activity on {c.D()}. Call {_phone(c)}.",
        f"Card {c.CARD()} unblocked. You can use it again.{c.noise()}",
        f"CARD {c.CARD()} BLOCKED {c.D()}. CALL {_phone(c)}"), split="negative"),
    Family("neg_en_promo", "en", "unknown", lambda c: c.pick(
        f"Get {_pct(c)}% cashback at {c.M()} until {c.D()}! Spend {c.AMT()} or more and win a trip.",
        f"{c.M()}: special offer! {_pct(c)}% off all purchases until {c.D()}. Pay with card {c.CARD()}.",
        f"Earn double points at {c.M()}, {c.C()} this weekend. Minimum spend {c.AMT()}.{c.noise()}",
        f"Cashback {c.AMT()} will be credited for purchases at {c.M()} made before {c.D()}."),
        split="negative", cases=("upper", "title")),
    Family("neg_en_limit", "en", "unknown", lambda c: c.pick(
        f"The daily limit on card {c.CARD()} has been changed to {c.AMT()}.",
        f"Your monthly spending limit is now {c.AMT()}. Changed on {c.D()}.{c.noise()}",
        f"Card {c.CARD()}: new cash withdrawal limit {c.AMT()} from {c.D()}."), split="negative"),
    Family("neg_en_balance", "en", "unknown", lambda c: c.pick(
        f"{_bal_en(c)} on card {c.CARD()} as of {c.D()}: {c.BAL()}.",
        f"{_bal_en(c)}: {c.BAL()}. Card {c.CARD()}. {c.D()}{c.noise()}",
        f"Statement for {c.D()}: {_bal_en(c).lower()} {c.BAL()}, card {c.CARD()}."), split="negative"),
    Family("neg_en_declined", "en", "unknown", lambda c: c.pick(
        f"Transaction declined at {c.M()}, {c.C()}: {c.AMT()}, card {c.CARD()}. Reason: wrong PIN.",
        f"Payment of {c.AMT()} at {c.M()} was not completed. Card {c.CARD()}. {c.D()}",
        f"DECLINED {c.AMT()} {c.M()} CARD{c.CARD()} {c.D()} - CARD EXPIRED",
        f"Purchase {c.AMT()} at {c.M()} rejected: limit reached. Card {c.CARD()}."), split="negative"),
    Family("neg_en_vercode", "en", "otp", lambda c: c.pick(
        f"Your verification number is {_digits(c)}. Do not share it with anyone.",
        f"{_digits(c)} is your confirmation number for the payment of {c.AMT()} at {c.M()}.",
        f"Use {_digits(c)} to confirm the login. Valid for 5 minutes.{c.noise()}"), split="negative"),
    Family("neg_ru_blocked", "ru", "unknown", lambda c: c.pick(
        f"Карта {c.CARD()} заблокирована. Для разблокировки позвоните {_phone(c)}.",
        f"Карта {c.CARD()} разблокирована.{c.noise()}",
        f"{c.D()} карта {c.CARD()} временно заблокирована. Телефон {_phone(c)}"), split="negative"),
    Family("neg_ru_login", "ru", "unknown", lambda c: c.pick(
        f"Вход в мобильный банк {c.D()}. Если это были не вы, позвоните {_phone(c)}.",
        f"Выполнен вход в интернет-банк с нового устройства {c.D()}.{c.noise()}"), split="negative"),
    Family("neg_ru_tariff", "ru", "unknown", lambda c: c.pick(
        f"С {c.D()} стоимость обслуживания карты {c.CARD()} составит {c.AMT()} в месяц.",
        f"Уважаемый клиент, тарифы меняются с {c.D()}. Подробнее на сайте банка.",
        f"Напоминаем: плата за смс-информирование {c.AMT()} будет списана {c.D()}."), split="negative"),
    Family("neg_ru_transfer_req", "ru", "unknown", lambda c: c.pick(
        f"Вам поступил запрос на перевод {c.AMT()} от {c.M()}. Подтвердите в приложении.",
        f"{c.M()} просит перевести {c.AMT()}. Ответьте в приложении до {c.D()}."), split="negative"),
    Family("neg_tr_promo", "tr", "unknown", lambda c: c.pick(
        f"Keshbek {_pct(c)}% v {c.M()} do {c.D()}! Oplachivayte kartoy {c.CARD()}.",
        f"Skidka {_pct(c)}% v {c.M()}, {c.C()} pri pokupke ot {c.AMT()}.{c.noise()}"), split="negative"),
    Family("neg_tr_parol", "tr", "otp", lambda c: c.pick(
        f"Parol dlya vhoda: {_digits(c)}. Nikomu ne soobshchayte.",
        f"Kod podtverzhdeniya platezha {c.AMT()} v {c.M()}: {_digits(c)}."), split="negative"),
    Family("neg_tr_limit", "tr", "unknown", lambda c: c.pick(
        f"Limit po karte {c.CARD()} izmenen: {c.AMT()}.",
        f"Ustanovlen novyy limit {c.AMT()} na snyatie nalichnyh s {c.D()}."), split="negative"),
    # ---- held out
    Family("neg_en_login", "en", "unknown", lambda c: c.pick(
        f"New sign-in to your account from {c.pick('iPhone', 'Android', 'Windows PC')} on {c.D()}. "
        f"Not you? Call {_phone(c)}.",
        f"Security alert: password changed on {c.D()}. If it was not you, contact us at {_phone(c)}."),
        heldout=True, split="negative"),
    Family("neg_en_p2p_request", "en", "unknown", lambda c: c.pick(
        f"{c.M()} requests {c.AMT()} from you. Open the app to accept or decline.",
        f"Money request: {c.AMT()} from {c.M()}, expires {c.D()}."), heldout=True, split="negative",
        cases=("upper", "title")),
    Family("neg_ru_promo", "ru", "unknown", lambda c: c.pick(
        f"Кэшбэк {_pct(c)}% в {c.M()} до {c.D()}! Оплачивайте картой {c.CARD()}.",
        f"Скидка {_pct(c)}% в {c.M()}, {c.C()} при покупке от {c.AMT()}."), heldout=True, split="negative"),
    Family("neg_ru_declined", "ru", "unknown", lambda c: c.pick(
        f"Отказ: операция {c.AMT()} в {c.M()}, {c.C()} не выполнена. Карта {c.CARD()}.",
        f"Покупка {c.AMT()} в {c.M()} отклонена. Карта {c.CARD()}. {c.D()}"), heldout=True, split="negative"),
    Family("neg_tr_blocked", "tr", "unknown", lambda c: c.pick(
        f"Karta {c.CARD()} zablokirovana. Dlya razblokirovki pozvonite {_phone(c)}.",
        f"Karta {c.CARD()} razblokirovana {c.D()}."), heldout=True, split="negative"),
)
# Procedural non-transactions (training only): a concept phrase from the language's pool --
# the same words the held-out negative families use, as the format families share their
# label words -- with a random subset of transaction-looking values (card, amount, date,
# merchant, phone, digits) in a random order and separators.  A held-out negative family
# is a NEW PHRASING of a concept whose words were trained on, never unseen vocabulary.
_NEG_CONCEPTS = {
    "en": {
        "blocked": ("card blocked", "card has been blocked", "card temporarily blocked", "card unblocked",
                    "card is locked", "BLOCKED", "account blocked"),
        "login": ("new sign-in", "login to online banking", "password changed", "security alert",
                  "new device login", "sign-in attempt"),
        "promo": ("cashback {pct}%", "{pct}% off", "special offer", "double points", "bonus offer", "win a trip"),
        "limit": ("limit changed", "new daily limit", "spending limit updated", "withdrawal limit"),
        "balance": ("balance as of", "statement", "balance info", "available balance notice"),
        "declined": ("declined", "transaction declined", "payment rejected", "not completed", "operation failed"),
        "p2p": ("money request", "requests money", "transfer request", "awaiting your confirmation"),
        "tariff": ("service fee", "tariff change", "monthly fee will be charged", "fees change"),
        "otp": ("verification number", "confirmation number", "one-time number", "security number"),
    },
    "ru": {
        "blocked": ("карта заблокирована", "карта разблокирована", "временно заблокирована", "блокировка карты"),
        "login": ("вход в мобильный банк", "вход в интернет-банк", "пароль изменен", "новое устройство"),
        "promo": ("кэшбэк {pct}%", "скидка {pct}%", "акция", "бонусы x2", "специальное предложение"),
        "limit": ("лимит изменен", "новый лимит", "лимит по карте"),
        "balance": ("баланс на", "остаток на", "выписка"),
        "declined": ("отказ", "операция отклонена", "не выполнена", "операция не прошла"),
        "p2p": ("запрос на перевод", "просит перевести", "ожидает подтверждения"),
        "tariff": ("плата за обслуживание", "тарифы меняются", "комиссия составит"),
        "otp": ("пароль для входа", "код подтверждения", "одноразовый пароль"),
    },
    "tr": {
        "blocked": ("karta zablokirovana", "karta razblokirovana", "vremenno zablokirovana", "blokirovka karty"),
        "login": ("vhod v mobilnyy bank", "parol izmenen", "novoe ustroystvo"),
        "promo": ("keshbek {pct}%", "skidka {pct}%", "aktsiya", "bonusy x2"),
        "limit": ("limit izmenen", "novyy limit", "limit po karte"),
        "balance": ("balans na", "ostatok na", "vypiska"),
        "declined": ("otkaz", "operatsiya otklonena", "ne vypolnena"),
        "p2p": ("zapros na perevod", "prosit perevesti"),
        "tariff": ("plata za obsluzhivanie", "tarify menyayutsya"),
        "otp": ("parol dlya vhoda", "kod podtverzhdeniya"),
    },
}
_NEG_LABELS = {"en": dict(card=("card", "Card"), amt=("Amount", "Sum"), date=("Date", "on"), phone=("Call", "Tel")),
               "ru": dict(card=("Карта", "карта"), amt=("Сумма",), date=("Дата",), phone=("Тел", "звоните")),
               "tr": dict(card=("Karta", "karta"), amt=("Summa",), date=("Data",), phone=("Tel", "zvonite"))}


def _neg_proc_render(c: _Ctx) -> str:
    r, lang = c.r, c.fam.lang
    concept = r.choice(tuple(_NEG_CONCEPTS[lang]))
    c.neg_txn = "otp" if concept == "otp" else "unknown"
    phrase = r.choice(_NEG_CONCEPTS[lang][concept]).format(pct=_pct(c))
    if r.random() < 0.5:
        phrase = phrase[0].upper() + phrase[1:]
    L = _NEG_LABELS[lang]
    vals = []
    if r.random() < 0.6:
        vals.append((r.choice(L["card"]) + " " if r.random() < 0.7 else "") + c.CARD())
    if r.random() < 0.55 or concept in ("promo", "limit", "balance", "declined", "p2p", "tariff"):
        v = c.BAL() if concept == "balance" else c.AMT()
        vals.append((r.choice(L["amt"]) + ": " if r.random() < 0.4 else "") + v)
    if r.random() < 0.55:
        vals.append((r.choice(L["date"]) + " " if r.random() < 0.4 else "") + c.D())
    if r.random() < 0.5 or concept in ("promo", "declined", "p2p"):
        vals.append(c.M() + (", " + c.C() if r.random() < 0.4 else ""))
    if concept == "otp" or r.random() < 0.15:
        vals.append(_digits(c))
    if concept in ("blocked", "login") and r.random() < 0.5:
        vals.append(r.choice(L["phone"]) + " " + _phone(c))
    r.shuffle(vals)
    k = r.randint(0, len(vals))
    segs = vals[:k] + [phrase] + vals[k:]
    # hard negatives: a transaction header word ("Purchase", "Покупка", "Oplata") in front
    # of a message the concept phrase makes a non-transaction (a declined purchase, a
    # payment request, a promo) -- the header alone never decides
    if concept in ("declined", "p2p", "promo", "tariff", "otp", "limit") and r.random() < 0.35:
        segs.insert(0, r.choice(_PROC_POOLS[lang]["head_debit"] + _PROC_POOLS[lang]["head_credit"]))
    sep = r.choice((", ", "; ", ". ", " ", " | ", "\n"))
    return sep.join(segs) + (c.noise() if sep != "\n" else "")


NEG_FAMILIES = NEG_FAMILIES + (
    Family("neg_proc_en", "en", "unknown", _neg_proc_render, split="negative", cases=("upper", "upper", "title")),
    Family("neg_proc_ru", "ru", "unknown", _neg_proc_render, split="negative"),
    Family("neg_proc_tr", "tr", "unknown", _neg_proc_render, split="negative"),
)
NEG_TRAIN_FAMILIES: Tuple[str, ...] = tuple(f.name for f in NEG_FAMILIES if not f.heldout)
NEG_HELDOUT_FAMILIES: Tuple[str, ...] = tuple(f.name for f in NEG_FAMILIES if f.heldout)
VALUE_HELDOUT_FAMILIES: Tuple[str, ...] = tuple(f.name for f in VALUE_FAMILIES)
_BY_NAME = {f.name: f for f in FAMILIES + VALUE_FAMILIES + NEG_FAMILIES}
# the reference's real-world formats are families too (training; up-weighted: they carry
# the golden CASES)
LEGACY_FAMILIES = ("legacy_purchase", "legacy_account", "legacy_credit")
TRAIN_FAMILIES: Tuple[str, ...] = LEGACY_FAMILIES + tuple(f.name for f in FAMILIES if not f.heldout)
HELDOUT_FAMILIES: Tuple[str, ...] = tuple(f.name for f in FAMILIES if f.heldout)
_LEGACY_WEIGHT = 3
_PROC_WEIGHT = 3  # procedural layouts: the training data's diversity


_SELECTORS = {
    "train": lambda: TRAIN_FAMILIES,
    "heldout": lambda: HELDOUT_FAMILIES,
    "all": lambda: TRAIN_FAMILIES + HELDOUT_FAMILIES,
    "heldout_values": lambda: VALUE_HELDOUT_FAMILIES,
    "neg_train": lambda: NEG_TRAIN_FAMILIES,
    "neg_heldout": lambda: NEG_HELDOUT_FAMILIES,
    "neg_all": lambda: NEG_TRAIN_FAMILIES + NEG_HELDOUT_FAMILIES,
}
# the non-transaction families mixed into a transaction selector (generate(negatives=p))
_NEG_OF = {"train": "neg_train", "heldout": "neg_heldout", "all": "neg_all", "heldout_values": "neg_heldout"}
NEGATIVE_TXN = ("unknown", "otp")


def family_names(which: Union[str, Sequence[str]]) -> Tuple[str, ...]:
    if isinstance(which, str):
        sel = _SELECTORS.get(which)
        return sel() if sel is not None else (which,)
    return tuple(which)


def is_negative(family: str) -> bool:
    f = _BY_NAME.get(family)
    return f is not None and f.split == "negative"


def rejection_answer(txn: str = "unknown") -> Dict[str, Optional[str]]:
    """The answer of a non-transaction: Gemini's shape with null fields."""
    return dict(txn_type=txn, date=None, amount=None, currency=None, card=None, merchant=None, city=None,
                address=None, balance=None)


def _family_one(r: random.Random, v: Vocab, name: str, all_credit_kinds: bool = False) -> SynthSMS:
    ts = r.randint(1_690_000_000, 1_750_000_000)
    if name in LEGACY_FAMILIES:
        cur, card = r.choice(_CURRENCIES), f"{r.randint(0, 9999):04d}"
        if name == "legacy_credit":
            # traffic: the kind the worker's keyword filter lets through to the LLM; training
            # also sees the skipped kinds (CREDIT PAYMENT / C2C RECEIVED: the legacy mix scores them)
            return _legacy_credit(r, ts, cur, card, kinds=None if all_credit_kinds else ("TRANSFER IN",))
        return (_legacy_purchase if name == "legacy_purchase" else _legacy_account)(r, v, ts, cur, card)
    fam = _BY_NAME[name]
    c = _Ctx(r, v, fam, ts)
    body = fam.render(c)
    if fam.split == "negative":
        return SynthSMS(body, "negative", rejection_answer(getattr(c, "neg_txn", fam.txn)), ts, name, None)
    exp = dict(c.exp)
    return SynthSMS(body, "purchase" if fam.txn == "debit" else "credit", dict(c.ans), ts, name, exp)


# traffic mixes (bench.py --traffic): "mixed" = every legacy kind in its natural share (17 %
# are skipped by the parser's keyword filter and never reach the LLM); "purchase" = the two
# legacy debit formats only (the BASELINE harness timed purchase bodies only); "formats" =
# every template family (train and held-out layouts, all LLM-routed); "heldout_formats" =
# the held-out families only
TRAFFIC: Dict[str, Dict[str, Any]] = {
    "mixed": {},
    "purchase": {"kinds": ("purchase", "account")},
    # every template family plus 10 % non-transactions: bank SMS
    # that pass the keyword filter and must end in the DLQ, not in sms.parsed
    "formats": {"families": "all", "negatives": 0.10},
    "heldout_formats": {"families": "heldout"},
}
TRAFFIC_KINDS = {k: v.get("kinds") for k, v in TRAFFIC.items() if "families" not in v}


def generate(n: int, seed: int = 0, unique: bool = True, vocab_name: str = "train",
             kinds: Optional[Sequence[str]] = None,
             families: Union[None, str, Sequence[str]] = None, training: bool = False,
             negatives: float = 0.0) -> List[SynthSMS]:
    """``n`` messages; with ``unique`` every body is distinct (defeats the response cache).
    ``vocab_name``: ``"train"`` (what the extractor is trained on) or ``"heldout"`` —
    merchant / city / street names disjoint from the training pools (held-out scoring
    and the benchmark's traffic).  ``kinds``: keep only these message kinds.
    ``families``: None = the legacy mix; else draw each message from these template
    families (``"train"``, ``"heldout"``, ``"all"``, ``"heldout_values"``,
    ``"neg_train"`` / ``"neg_heldout"`` / ``"neg_all"`` or names), uniformly by family with
    the legacy formats and the procedural layouts weighted x3 in ``"train"`` / ``"all"``.
    ``negatives``: the share of messages drawn from the non-transaction families of the
    same split (``"train"`` -> ``"neg_train"`` ...).
    ``training``: also the legacy credit kinds the keyword filter skips (never traffic)."""
    r = random.Random(seed)
    v = vocab(vocab_name)
    names: Tuple[str, ...] = ()
    weights: List[int] = []
    neg_names: Tuple[str, ...] = ()
    if families is not None:
        names = family_names(families)
        # SMSGATE_PROC_WEIGHT: training-mix experiments (scripts/qa_probe.py --variants)
        pw = int(os.environ.get("SMSGATE_PROC_WEIGHT", _PROC_WEIGHT))
        weights = [(_LEGACY_WEIGHT if f in LEGACY_FAMILIES else pw if f.startswith("proc_") else 1)
                   if len(names) > 3 else 1 for f in names]
        if negatives > 0:
            if not isinstance(families, str) or families not in _NEG_OF:
                raise ValueError(f"negatives need a split selector ({sorted(_NEG_OF)}), not {families!r}")
            neg_names = family_names(_NEG_OF[families])
            neg_weights = [_PROC_WEIGHT if f.startswith("neg_proc_") else 1 for f in neg_names]
    out: List[SynthSMS] = []
    seen = set()
    while len(out) < n:
        if not names:
            s = _one(r, v)
        elif neg_names and r.random() < negatives:
            s = _family_one(r, v, r.choices(neg_names, neg_weights)[0], training)
        else:
            s = _family_one(r, v, r.choices(names, weights)[0], training)
        if kinds is not None and s.kind not in kinds:
            continue
        if unique:
            if s.body in seen:
                continue
            seen.add(s.body)
        out.append(s)
    return out


def generate_traffic(n: int, seed: int = 0, vocab_name: str = "heldout", traffic: str = "mixed") -> List[SynthSMS]:
    """Bench / evaluation traffic by preset name (:data:`TRAFFIC`)."""
    return generate(n, seed=seed, vocab_name=vocab_name, **TRAFFIC[traffic])


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
    (``"tokenizer"`` vocabulary: real training-split words only; the legacy mix and
    the TRAINING template families — held-out layouts contribute no merges)."""
    from ..parse.text import normalize_body

    half = n // 2
    items = generate(half, seed, unique=False, vocab_name="tokenizer") + \
        generate(n - half, seed + 1, unique=False, vocab_name="tokenizer", families="train")
    for s in items:
        yield s.body
        yield normalize_body(s.body)
        if s.answer:
            yield " ".join(v for v in s.answer.values() if v)
