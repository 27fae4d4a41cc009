"""The native per-message parse path (native/csrc/parsefast.cpp, parse/fastpath.py)
against the Python path it replaces, byte for byte.

Whenever the native code answers -- a scanned RawSMS, an sms.parsed payload, an
unmatched verdict -- the Python path must give exactly that; every other case must be
handed back (None / FALLBACK).  Checked on the synthetic corpus (every template family,
legacy kinds, non-transactions), on mutated answers (dates, amounts, currencies, cards
of every shape the grammar and a model can produce) and on hostile JSON / strings."""
from __future__ import annotations

import json
import random
from datetime import datetime, timedelta

import pytest

from smsgate_amd.models.domain import RawSMS, parsed_wire
from smsgate_amd.parse import fastpath
from smsgate_amd.parse.canonical import canonical_date_text
from smsgate_amd.parse.dates import parse_custom_datetime
from smsgate_amd.parse.numeric import parse_ambiguous_decimal
from smsgate_amd.parse.pipeline import Outcome, postprocess_answer
from smsgate_amd.parse.text import llm_should_skip, normalize_body, worker_should_skip
from smsgate_amd.serving.qa import null_rejection
from smsgate_amd.utils import synth

pytestmark = pytest.mark.skipif(not fastpath.available(), reason="_parsefast not built")

FIELDS = ("txn_type", "date", "amount", "currency", "card", "merchant", "city", "address", "balance")


def _corpus(n=3000, seed=1):
    items = synth.generate_traffic(n, seed=seed, traffic="formats")
    items += synth.generate(n // 3, seed=seed + 1, vocab_name="heldout")  # legacy kinds: OTP, C2C ...
    items += synth.generate(n // 3, seed=seed + 2, vocab_name="heldout", families="heldout_values")
    return items


def _payload(i, s, r):
    d = {"msg_id": f"m{i}", "sender": r.choice(["BANK", "ACBA", "Банк"]), "body": s.body, "date": str(s.timestamp),
         "device_id": r.choice(["dev-1", None]), "source": r.choice(["device", "xml"])}
    if r.random() < 0.1:
        del d["device_id"]
    if r.random() < 0.1:
        del d["source"]
    if r.random() < 0.1:
        d["extra"] = r.choice([1, "x", None, [1, {"a": "b"}], True])
    return json.dumps(d, ensure_ascii=r.random() < 0.5).encode()


def _python_raw(data: bytes):
    """The parser's Python path: (RawSMS | None, skipped?)."""
    try:
        raw = RawSMS.model_validate_json(data)
    except Exception:
        return None, None
    return raw, worker_should_skip(raw.body) or llm_should_skip(raw.body)


def test_scan_equals_pydantic_and_the_keyword_filters():
    r = random.Random(3)
    items = _corpus()
    payloads = [_payload(i, s, r) for i, s in enumerate(items)]
    got = fastpath.scan(payloads)
    fast = 0
    for data, fr in zip(payloads, got):
        raw, skipped = _python_raw(data)
        if fr is None:
            continue
        fast += 1
        assert raw is not None and not skipped, data
        assert fr.model_dump() == raw.model_dump(), data
        assert fr.norm == normalize_body(raw.body)
    assert fast > 0.8 * len(payloads), (fast, len(payloads))
    # skipped kinds (OTP, C2C ...) are never taken by the native scan
    assert all(g is None for g, s in zip(got, items) if s.kind in ("otp", "funds"))


def test_scan_hostile_json_never_disagrees():
    r = random.Random(4)
    base = [_payload(i, s, r) for i, s in enumerate(_corpus(300, seed=5))]
    variants = [
        b'{"msg_id":"a","sender":"B","body":"x","date":"1"}', b'{"msg_id":"a","sender":"","body":"x","date":"1"}',
        b'{"msg_id":1,"sender":"B","body":"x","date":"1"}', b'{"msg_id":"a","sender":"B","body":"x"}',
        b'{"msg_id":"a","sender":"B","body":"x","date":"1","source":"web"}', b'[1,2]', b'null', b'',
        b'{"msg_id":"a","sender":"B","body":"x","date":"1","msg_id":"b"}', b'{"raw":{"msg_id":"a"}}',
        b'{"msg_id":"a","sender":"B","body":"\\ud800","date":"1"}', b'{"msg_id":"a","sender":"B","body":"\\ud83d\\ude00",'
        b'"date":"1"}', b'{"msg_id":"a","sender":"B","body":"x\ny","date":"1"}', b'\xef\xbb\xbf{"msg_id":"a"}',
        b'{"msg_id":"a","sender":"B","body":"x","date":"1","n":1e999}', b'{"msg_id":"a","sender":"B","body":"x",'
        b'"date":"1","n":12345678901234567890}', b'{"msg_id":"a","sender":"B","body":"caf\xc3\xa9 \xe2\x80\xa2 ***",'
        b'"date":"1"} ', b'{"msg_id":"a","sender":"B","body":"Stra\xc3\x9fe OTP","date":"1"}',
        b'{"msg_id":"a","sender":"B","body":"ROTP","date":"1"}', b'{"msg_id":"a","sender":"B","body":"\xd9\xa1\xd9\xa2",'
        b'"date":"1"}', b'{"msg_id":"a","sender":"B","body":"1234***5678 x","date":"1","device_id":null}',
        b'{"msg_id":"a","sender":"B","body":"x","date":"1","device_id":7}', b'{"msg_id":"a","sender":"B","body":"x",'
        b'"date":"1"}}', b'{"msg_id":"a" , "sender" : "B","body":"\\u0041\\n\\t","date":"1"}',
    ]
    for b in base[:200]:  # random byte mutations
        for _ in range(3):
            k = r.randrange(len(b))
            variants.append(b[:k] + bytes([r.randrange(256)]) + b[k + 1:])
            variants.append(b[:k] + b[k + 1:])
    got = fastpath.scan(variants)
    for data, fr in zip(variants, got):
        if fr is None:
            continue
        raw, skipped = _python_raw(data)
        assert raw is not None and not skipped and fr.model_dump() == raw.model_dump(), data
        assert fr.norm == normalize_body(raw.body)


def _mutations(r, s):
    """Answers a model can produce for ``s``: the gold one and edits of single fields."""
    a = dict(s.answer) if s.answer else dict.fromkeys(FIELDS, "")
    out = [a]
    for _ in range(3):
        b = dict(a)
        f = r.choice(FIELDS)
        b[f] = r.choice([
            "", " ", "null", "None", "-", ".", "1,000", "1.234.567", "-52.00", "0.0000001", "5.", ".5", "1 234,56",
            "12'345.67", "USD", "usd.", "$", "руб", "Руб.", "драм", "₽", "€", "x", "*", "**12", "0018", "12345678",
            "4083***7538", "06.05.25 14:23", "31.02.2025 10:00", "2025-13-01", "Jun 6, 2025 2:23 PM", "6 June 2025",
            "14:23 6 июня 2025", "6 июня 2025 в 14:23", "6 июня 2025 г. 14:23", "6 ИЮНЯ 2025 Г. 14:23",
            "6  iyunya 2025", "6 iyunya 2025 v 14:23", "22 марта 2025", "2:20 AM 08.10.2024", "13:00 PM 01.01.2024",
            "2099-01-01 10:00", "01/02/2023 3:04pm", "debit", "credit", "otp", "unknown", "DEBIT", "Ä", "ß",
            " USD", "1 234,56", "١٢٣", "TEST \"LLC\"\n\\", "\x01\x1f\x7f", "😀",
            (a.get(f) or "") + " ", (a.get(f) or "")[:3],
        ])
        out.append(b)
    return out


def test_postprocess_equals_the_python_path_byte_for_byte():
    r = random.Random(7)
    items = _corpus(2400, seed=9)
    rows, raws, answers = [], [], []
    for i, s in enumerate(items):
        payload = _payload(i, s, r)
        fr = fastpath.scan([payload])[0]
        if fr is None:
            continue
        for a in _mutations(r, s):
            rows.append([a.get(f) if a.get(f) is not None else "" for f in FIELDS])
            raws.append(fr)
            answers.append(a)
    got = fastpath.postprocess(rows, raws)
    kinds = {"bytes": 0, fastpath.UNMATCHED: 0, fastpath.FALLBACK: 0}
    now = datetime.now()
    for row, fr, res in zip(rows, raws, got):
        ans = null_rejection(dict(zip(FIELDS, row)))
        py = postprocess_answer(fr, fr.norm, ans)
        if isinstance(res, bytes):
            kinds["bytes"] += 1
            assert py.outcome is Outcome.PARSED, (row, py)
            assert not py.parsed.date > now + timedelta(seconds=1)
            assert parsed_wire(py.parsed) == res, (row, res)
        elif res == fastpath.UNMATCHED:
            kinds[res] += 1
            assert py.outcome is Outcome.UNMATCHED, (row, py)
        else:
            assert res == fastpath.FALLBACK
            kinds[res] += 1
    assert kinds["bytes"] > 0.5 * len(rows) and kinds[fastpath.UNMATCHED] > 0 and kinds[fastpath.FALLBACK] > 0, kinds


def test_gold_answers_take_the_native_path():
    """The common case is native: every gold answer of the traffic parses there."""
    r = random.Random(8)
    items = [s for s in synth.generate_traffic(2000, seed=11, traffic="formats") if s.answer]
    frs = fastpath.scan([_payload(i, s, r) for i, s in enumerate(items)])
    pairs = [(s, fr) for s, fr in zip(items, frs) if fr is not None]
    assert len(pairs) > 0.95 * len(items)
    rows = [[null_rejection(s.answer).get(f) or "" for f in FIELDS] for s, _ in pairs]
    got = fastpath.postprocess(rows, [fr for _, fr in pairs])
    neg = sum(s.kind == "negative" for s, _ in pairs)
    native = sum(isinstance(g, bytes) for g in got) + sum(g == fastpath.UNMATCHED for g in got)
    assert sum(g == fastpath.UNMATCHED for g in got) == neg
    assert native >= 0.99 * len(pairs), (native, len(pairs))


def test_native_dates_and_decimals_fuzzed_against_python():
    from smsgate_amd.parse.fastpath import _ext, _now

    ext = _ext()
    r = random.Random(12)
    mons = ["Jun", "June", "jun", "Sept", "Foo", "июня", "июн", "Июня", "ИЮНЯ", "мая", "май", "iyunya", "Maya", "mart"]
    for _ in range(20000):
        y, a, b = r.randint(1990, 2030), r.randint(0, 32), r.randint(0, 32)
        hh, mi = r.randint(0, 24), r.randint(0, 60)
        sp = r.choice([" ", "  ", "", "\t"])
        mo = r.choice(mons)
        s = r.choice([
            f"{a:02d}.{b:02d}.{y % 100:02d} {hh:02d}:{mi:02d}", f"{y}-{a % 13:02d}-{b:02d}{r.choice([' ', 'T'])}{hh:02d}:{mi:02d}",
            f"{a:02d}.{b:02d}.{y}", f"{hh:02d}:{mi:02d} {a:02d}.{b:02d}.{y}", f"{a}{r.choice([' ', '-'])}{mo}{sp}{y}",
            f"{a}/{b}/{y}{sp}{hh}:{mi:02d}", f"{a:02d}-{b:02d}-{y % 100:02d}", f"{a} {mo} {y}{sp}г.{sp}{hh}:{mi:02d}",
            f"{a} {mo}. {y} в {hh}:{mi:02d}", f"{hh}:{mi:02d}{sp}{a} {mo} {y}", f"{mo} {a}, {y} {hh}:{mi:02d}{sp}PM",
            f"{hh}:{mi:02d} am {a:02d}.{b:02d}.{y}", f"{a} {mo} {y} v {hh}:{mi:02d}", f"{a}{sp}{mo}{sp}{y}",
            f"{a:02d}.{b:02d}.{y} {hh}:{mi:02d}{sp}pm", f" {a:02d}.{b:02d}.{y} ", f"{a}/{b}/{y}{r.choice(['0', 'x', ''])}",
        ])
        want_text = canonical_date_text(s)
        try:
            want = parse_custom_datetime(want_text)
        except Exception:
            want = None
        text, t = ext.canonical_date(s, _now())
        if text is not None:
            assert text == want_text, (s, text, want_text)
        if t is not None:
            assert want == datetime(*t), (s, t, want)
    for _ in range(20000):
        v = "".join(r.choice("0123456789.,- '+eE_x") for _ in range(r.randint(0, 9)))
        try:
            want = str(parse_ambiguous_decimal(v))
        except Exception:
            want = None
        got = ext.decimal(v)
        if got is not None:
            assert got == want, (v, got, want)


def test_normalize_equals_python():
    from smsgate_amd.parse.fastpath import _ext

    ext = _ext()
    r = random.Random(13)
    for _ in range(5000):
        s = "".join(r.choice("0123*4 • ab") for _ in range(r.randint(0, 30)))
        assert ext.normalize(s) == normalize_body(s), s


class _RowBackend:
    """A backend answering from a table (normalised body -> answer row), as dict answers
    (extract_batch) or rows (extract_rows, the native path's interface); one body raises."""
    name = "table"
    max_batch = 512

    def __init__(self, table):
        self.table = table

    async def extract_batch(self, bodies):
        out = []
        for b in bodies:
            row = self.table.get(b)
            out.append(RuntimeError("backend failed") if row is None else null_rejection(dict(zip(FIELDS, row))))
        return out

    async def extract_rows(self, bodies):
        return [RuntimeError("backend failed") if self.table.get(b) is None else list(self.table[b]) for b in bodies]

    async def start(self):
        pass

    async def close(self):
        pass


def test_route_batch_is_byte_identical_with_and_without_the_native_path(arun, monkeypatch):
    """The parser's whole output (every sms.parsed / sms.processing payload, every DLQ
    envelope shape, the counters) with the native path on equals the Python path's,
    message for message: gold and mutated answers, non-transactions, keyword skips,
    invalid payloads, backend errors, cards too short (BROKEN), future dates."""
    from smsgate_amd.bus.base import Msg
    from smsgate_amd.parse.pipeline import ParsePipeline
    from smsgate_amd.services.parser import route_batch

    r = random.Random(21)
    items = _corpus(900, seed=22)
    table, payloads = {}, []
    for i, s in enumerate(items):
        p = _payload(i, s, r)
        a = r.choice(_mutations(r, s))
        if r.random() < 0.05:
            a = dict(a, date=(datetime.now() + timedelta(days=30)).strftime("%d.%m.%Y %H:%M"))  # future
        if r.random() < 0.05:
            a = dict(a, card="12")  # BROKEN
        if r.random() > 0.03:  # else: the backend raises for this body
            table[normalize_body(s.body)] = [a.get(f) if a.get(f) is not None else "" for f in FIELDS]
        payloads.append(p)
    payloads += [b"not json", b'{"msg_id":"x"}', b'{"raw":' + payloads[0] + b'}', b'{"msg_id":"q","sender":"B",'
                 b'"body":"Your OTP code: 123","date":"1"}']

    from smsgate_amd.bus.base import MsgMetadata

    def run(pipe=None):
        pipe = pipe or ParsePipeline(_RowBackend(table))
        msgs = [Msg("sms.raw", d, MsgMetadata(i, 1, 0.0, "SMS", "t"), None) for i, d in enumerate(payloads)]
        return arun(route_batch(pipe, msgs))

    native_out, native_counts = run()
    # a replay answered from the response cache (rows cached as the nine decoded strings,
    # turned into the answer dict on the Python path) routes every message the same way
    pipe = ParsePipeline(_RowBackend(table))
    run(pipe)
    pipe.backend.table = {}  # every answer must now come from the cache
    replay_out, replay_counts = run(pipe)
    assert replay_counts == native_counts
    assert [x for x, _ in replay_out] == [x for x, _ in native_out]
    assert [b for x, b in replay_out if x != "sms.failed"] == [b for x, b in native_out if x != "sms.failed"]
    monkeypatch.setattr(fastpath, "_EXT", None)
    monkeypatch.setattr(fastpath, "_TRIED", True)
    py_out, py_counts = run()
    assert native_counts == py_counts
    assert len(native_out) == len(py_out)
    for (sa, a), (sb, b) in zip(native_out, py_out):
        assert sa == sb, (a, b)
        if sa == "sms.failed":  # the envelopes: same shape and content (err texts may differ in wording)
            ja, jb = json.loads(a), json.loads(b)
            assert ja.keys() == jb.keys() and ja.get("raw") == jb.get("raw") and ja.get("entry") == jb.get("entry")
            assert ja.get("reason") == jb.get("reason")
        else:
            assert a == b
    assert native_counts["parsed"] > 300 and native_counts["fail"] > 50, native_counts


def test_raw_wires_equal_the_gateway_mapping():
    """The gateway role's sms.raw payloads (bench ingestion): native md5 id + RawSMS
    JSON == raw_wire(payload_to_raw(p)); payloads RawSMS refuses raise as before."""
    from smsgate_amd.models.domain import raw_wire
    from smsgate_amd.services.gateway import RawSMSPayload, payload_to_raw

    r = random.Random(31)
    ps = [RawSMSPayload(device_id=r.choice(["bench", "dev \"x\"\n", "Д"]), message=s.body, sender=r.choice(["BANK", "Банк"]),
                        timestamp=r.choice([s.timestamp, -5, 0, 10 ** 15]), source=r.choice(["device", "xml"]))
          for s in _corpus(600, seed=32)]
    ps += [RawSMSPayload(device_id="d", message="x\x00\x1f\x7f😀 ", sender="s", timestamp=1, source="device")]
    assert fastpath.raw_wires(ps) == [raw_wire(payload_to_raw(p)) for p in ps]
    for bad in (RawSMSPayload(device_id="d", message="", sender="s", timestamp=1, source="device"),
                RawSMSPayload(device_id="d", message="m", sender="s", timestamp=1, source=None),
                RawSMSPayload(device_id="d", message="m", sender="s", timestamp=1, source="web")):
        with pytest.raises(Exception):
            fastpath.raw_wires([bad])


def test_writer_peek_accepts_only_valid_parsed_payloads():
    """The writer's native check: whenever it accepts a payload, pydantic validates it to
    the same msg_id, merchant truthiness and date; payloads off the canonical form, or
    invalid, are left to pydantic.  And the writer's output (sink records, skips, DLQ)
    is the pydantic path's."""
    from decimal import Decimal

    from smsgate_amd.models.domain import ParsedSMS

    r = random.Random(41)
    good = []
    for s in _corpus(600, seed=42):
        if not s.answer or s.kind == "negative":
            continue
        raw = RawSMS(msg_id=f"m{len(good)}", sender="B", body=s.body, date=str(s.timestamp), device_id=r.choice(["d", None]))
        p = postprocess_answer(raw, normalize_body(s.body), s.answer).parsed
        if p is not None:
            good.append(parsed_wire(p))
    good.append(parsed_wire(ParsedSMS(msg_id="x", device_id=None, sender="s", date=datetime(2024, 2, 29, 1, 2, 3),
                                      raw_body="b", txn_type="otp", amount=None, currency=None, card=None,
                                      merchant="", city=None, address=None, balance=Decimal("-0.0"))))
    bad = []
    for g in good[:150]:
        for a, b in ((b'"date":"', b'"date":"2025-02-30T'), (b'"card":"', b'"card":"12345'), (b'"amount":"', b'"amount":"1E'),
                     (b'"txn_type":"', b'"txn_type":"x'), (b',"city"', b', "city"'), (b'"amount":"', b'"amount":'),
                     (b'{"msg_id"', b'{"msg_id":"y","msg_id"')):
            bad.append(g.replace(a, b, 1))
        k = r.randrange(len(g))
        bad.append(g[:k] + bytes([r.randrange(256)]) + g[k + 1:])
    allp = good + bad
    got = fastpath.peek_parsed(allp)
    assert all(g is not None for g in got[:len(good)])
    for data, pk in zip(allp, got):
        if pk is None:
            continue
        p = ParsedSMS.model_validate_json(data)
        assert pk[0] == p.msg_id and pk[1] == bool(p.merchant) and datetime(*pk[2]) == p.date, data


def test_pipeline_null_rejection_matches_the_engine_rule():
    from smsgate_amd.parse.pipeline import _REJECT_TXN, _null_rejection
    from smsgate_amd.serving.qa import REJECT_TXN

    assert tuple(_REJECT_TXN) == tuple(REJECT_TXN)
    for t in ("debit", "credit", "otp", "unknown"):
        a = dict(zip(FIELDS, [t] + ["x"] * 8))
        assert _null_rejection(a) == null_rejection(a)


@pytest.mark.parametrize("first", ["smsgate_amd.serving", "smsgate_amd.parse", "smsgate_amd.serving.qa",
                                   "smsgate_amd.parallel.replica", "smsgate_amd.services.parser"])
def test_package_imports_in_any_order(first):
    """A fresh interpreter imports every package whichever comes first (a parse ->
    serving import made serving-first imports circular)."""
    import subprocess
    import sys

    code = f"import {first}; import smsgate_amd.parse.pipeline, smsgate_amd.serving.remote, smsgate_amd.services.writer"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


def test_scan_record_carries_the_cache_key_and_fields():
    """A FastRaw's cache key is parse/cache.py cache_key of its normalised body, and the
    RawSMS fields read back from its native record are pydantic's."""
    from smsgate_amd.models.domain import RawSMS
    from smsgate_amd.parse.cache import cache_key

    r = random.Random(7)
    items = synth.generate(300, seed=61, vocab_name="heldout", families="all", negatives=0.1)
    payloads = [_payload(i, s, r) for i, s in enumerate(items)]
    got = fastpath.scan(payloads)
    assert sum(g is not None for g in got) > 250
    for p, g in zip(payloads, got):
        if g is None:
            continue
        ref = RawSMS.model_validate_json(p)
        assert g.key == cache_key(normalize_body(ref.body)) and g.norm == normalize_body(ref.body)
        assert g.model_dump() == ref.model_dump()
        assert (g.msg_id, g.sender, g.body, g.date, g.device_id, g.source) == (
            ref.msg_id, ref.sender, ref.body, ref.date, ref.device_id, ref.source)
