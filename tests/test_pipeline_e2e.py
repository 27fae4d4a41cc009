"""End-to-end slice: POST /sms/raw → bus → parser → sms.parsed → writer → sinks.

The reference's three parser CASES (tests/test_parsers.py:11-58) run through
the full pipeline with deterministic backends instead of live Gemini.
"""
import asyncio
import json
from datetime import datetime
from decimal import Decimal

import pytest
from fastapi.testclient import TestClient

from conftest import REFERENCE_CASES
from smsgate_amd.bus import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_RAW, MemoryBus
from smsgate_amd.models import RawSMS, TxnType
from smsgate_amd.parse import ParsePipeline
from smsgate_amd.parse.backends import FakeBackend, RegexBackend
from smsgate_amd.parse.backends.base import BackendError
from smsgate_amd.services.gateway import create_app
from smsgate_amd.services.parser import FUTURE_DATE_ERR, ParserWorker
from smsgate_amd.services.writer import WriterService
from smsgate_amd.sinks import MemorySink
from smsgate_amd.sinks.sql import SqlSink


def _raw(body, msg_id="test-msg-id", date="2025-05-06T00:00:00"):
    return RawSMS(msg_id=msg_id, device_id="test-device", sender="BANK", date=date, body=body, source="device")


@pytest.mark.parametrize("body, exp", REFERENCE_CASES)
def test_reference_cases_regex_backend(body, exp, arun):
    res = arun(ParsePipeline(RegexBackend()).parse(_raw(body)))
    p = res.parsed
    assert p is not None, res
    assert p.txn_type == TxnType.DEBIT
    assert (p.merchant, p.city, p.address, p.card, p.currency) == (
        exp["merchant"], exp["city"], exp["address"], exp["card"], exp["currency"])
    assert p.amount == Decimal(exp["amount"]) and p.balance == Decimal(exp["balance"])
    assert p.date == datetime(*exp["date"])


async def _drain(bus, subject):
    sub = await bus.subscribe(subject, "inspect-" + subject.replace(".", "-"))
    out = []
    while True:
        got = await sub.fetch(100, 0.05)
        if not got:
            return out
        for m in got:
            await m.ack()
            out.append(json.loads(m.data))


def test_full_pipeline_http_to_sql(tmp_path, arun):
    bus = MemoryBus()

    async def get_bus():
        return bus

    with TestClient(create_app(get_bus)) as c:
        for i, (body, _) in enumerate(REFERENCE_CASES):
            r = c.post("/sms/raw", json={"device_id": "dev", "message": body, "sender": "BANK",
                                         "timestamp": 1749808562 + i, "source": "device"})
            assert r.status_code == 202
        # non-transaction + unparsable messages
        c.post("/sms/raw", json={"device_id": "dev", "message": "Your OTP is 1234", "sender": "BANK",
                                 "timestamp": 1, "source": "device"})
        c.post("/sms/raw", json={"device_id": "dev", "message": "hello there", "sender": "BANK",
                                 "timestamp": 1, "source": "device"})

    mem = MemorySink()
    sql = SqlSink(f"sqlite:///{tmp_path/'db.sqlite'}")

    async def go():
        parser = ParserWorker(bus, ParsePipeline(RegexBackend()), stats_interval=0)
        writer = WriterService(bus, [mem, sql], retry_attempts=1, stats_interval=0)
        assert await parser.stage.run_until_idle() == 5
        assert await writer.stage.run_until_idle() == 3
        parsed = await _drain(bus, SUBJECT_PARSED)
        processing = await _drain(bus, SUBJECT_PROCESSING)
        failed = await _drain(bus, SUBJECT_FAILED)
        return parser, writer, parsed, processing, failed

    parser, writer, parsed, processing, failed = arun(go())
    assert parser.counts == {"ok": 4, "fail": 1, "skip": 0,  # OTP counted OK (D11 parity) ...
                             "parsed": 3, "keyword_skipped": 1}  # ... and reported apart
    assert len(parsed) == 3 and parsed == processing
    assert [f.get("reason") for f in failed] == ["unmatched"] and failed[0]["raw"]["body"] == "hello there"
    assert writer.ok == 3 and writer.fail == 0
    assert {r.merchant for r in mem.all()} == {"TEST LLC", "TEST", "AMERIABANK API GATE"}
    assert sql.count() == 3
    # idempotent: replaying the same parsed records does not duplicate rows
    arun(sql.upsert_many(mem.all()))
    assert sql.count() == 3


def test_parser_dlq_envelopes(arun):
    bus = MemoryBus()
    boom = {"boom body"}

    def fail(body):
        return BackendError("LLM exploded") if body in boom else None

    future = dict(FakeBackend().default, date="01.01.2099 10:00")
    backend = FakeBackend(answers={"future body": future, "nocard": dict(FakeBackend().default, card="***")},
                          fail=fail)

    async def go():
        await bus.publish(SUBJECT_RAW, b"{not json")
        await bus.publish(SUBJECT_RAW, _raw("boom body").model_dump_json().encode())
        await bus.publish(SUBJECT_RAW, _raw("future body").model_dump_json().encode())
        await bus.publish(SUBJECT_RAW, _raw("nocard").model_dump_json().encode())
        # a DLQ envelope with `raw` is unwrapped and re-parsed
        env = {"reason": "unmatched", "raw": _raw("fine body").model_dump()}
        await bus.publish(SUBJECT_RAW, json.dumps(env).encode())
        w = ParserWorker(bus, ParsePipeline(backend), stats_interval=0)
        await w.stage.run_until_idle()
        return w, await _drain(bus, SUBJECT_FAILED), await _drain(bus, SUBJECT_PARSED)

    w, failed, parsed = arun(go())
    assert w.counts == {"ok": 1, "fail": 3, "skip": 1, "parsed": 1, "keyword_skipped": 0}
    assert failed[0]["entry"] == "{not json" and "err" in failed[0]
    assert failed[1] == {"err": "LLM exploded", "entry": _raw("boom body").model_dump()}
    assert failed[2]["err"] == FUTURE_DATE_ERR
    assert len(parsed) == 1 and parsed[0]["raw_body"] == "fine body"


def test_handler_exception_does_not_kill_loop(arun):
    """D1: a crashing batch is nak'ed and redelivered; the loop keeps consuming."""
    bus = MemoryBus()
    calls = {"n": 0}

    async def go():
        w = ParserWorker(bus, ParsePipeline(FakeBackend()), stats_interval=0)
        w.stage.nak_delay = 0.0
        real = w.stage.handler

        async def flaky_handler(msgs):
            calls["n"] += 1
            if calls["n"] == 1:
                raise RuntimeError("handler bug")
            await real(msgs)

        w.stage.handler = flaky_handler
        await bus.publish(SUBJECT_RAW, _raw("x").model_dump_json().encode())
        await w.stage.run_until_idle(idle_s=0.2)
        return w

    w = arun(go())
    assert w.stage.handler_errors == 1 and calls["n"] == 2
    assert w.counts == {"ok": 1, "fail": 0, "skip": 0, "parsed": 1, "keyword_skipped": 0}


def test_parser_tracing_spans_and_sentry_forwarding(arun, monkeypatch):
    """The parser records the reference's transaction and spans
    (worker.py:33-55, :80-171) in the in-process tracer, and forwards them to
    the Sentry SDK when one is active (stub SDK here: sentry_sdk is not on the
    image). The DLQ Profiler drives the SDK's profiler the same way."""
    import contextlib

    from smsgate_amd.obs import errors
    from smsgate_amd.obs.tracing import Profiler, tracer

    seen = []

    class _Prof:
        def start_profiler(self):
            seen.append(("profiler", "start"))

        def stop_profiler(self):
            seen.append(("profiler", "stop"))

    class _SDK:
        profiler = _Prof()

        def start_transaction(self, op, name):
            seen.append(("txn", f"{op}/{name}"))
            return contextlib.nullcontext()

        def start_span(self, name):
            seen.append(("span", name))
            return contextlib.nullcontext()

    monkeypatch.setattr(errors, "_sdk", _SDK())
    monkeypatch.setattr(tracer, "enabled", True)
    tracer.reset()
    bus = MemoryBus()

    async def go():
        await bus.publish(SUBJECT_RAW, _raw("traced body").model_dump_json().encode())
        w = ParserWorker(bus, ParsePipeline(FakeBackend()), stats_interval=0)
        await w.stage.run_until_idle()
        return w

    w = arun(go())
    assert w.counts["ok"] == 1
    snap = tracer.snapshot()
    for name in ("task/process_parsing", "validate", "parsing", "validate_parsed", "publish"):
        assert snap[name].count >= 1 and snap[name].max_s >= snap[name].mean_s >= 0.0, name
    assert ("txn", "task/process_parsing") in seen
    assert {n for k, n in seen if k == "span"} >= {"validate", "parsing", "validate_parsed", "publish"}
    with Profiler("dlq_reparse", out_dir=""):
        pass
    assert seen[-2:] == [("profiler", "start"), ("profiler", "stop")]
    tracer.reset()
