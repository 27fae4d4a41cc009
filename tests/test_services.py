"""Service-level tests: XML watcher, DLQ re-parser, notifier, MCP tools server,
Gemini REST backend, webhook receiver, legacy batch tools, PocketBase client, CLI.

External HTTP services are faked in-process (tests/fakes.py) — the image has
no network; parity for the reference's live-service behaviour (Gemini output,
PocketBase server rules, Telegram delivery) is "parity unpinned" beyond the
request/response shapes asserted here.
"""
from __future__ import annotations

import asyncio
import json
from datetime import datetime, timedelta, timezone
from decimal import Decimal

import httpx
import pytest
from fastapi.testclient import TestClient

from conftest import REFERENCE_CASES, drain
from fakes import FakePocketBase, FakeTelegram
from smsgate_amd.bus import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_RAW, MemoryBus
from smsgate_amd.bus.base import SUBJECT_FAILED_FINAL
from smsgate_amd.models import ParsedSMS, RawSMS, get_sha1_hash
from smsgate_amd.parse import ParsePipeline
from smsgate_amd.parse.backends import RegexBackend
from smsgate_amd.parse.backends.base import BackendError
from smsgate_amd.parse.cache import SqliteKV


# --------------------------------------------------------------------------- XML watcher
def test_xml_watcher_imports_and_moves(tmp_path, arun):
    from smsgate_amd.services.xml_watcher import XmlWatcher, iter_sms, write_backup_xml

    body = REFERENCE_CASES[0][0]
    f = tmp_path / "sms-2025.xml"
    write_backup_xml(f, [("BANK", 1746541380000, body), ("Other", 1746541440000, "hello")])
    msgs = list(iter_sms(f))
    assert msgs[0].source == "xml" and msgs[0].device_id == "xml_backup"
    assert msgs[0].msg_id == get_sha1_hash(body) and msgs[0].sender == "BANK"
    assert msgs[0].date == datetime.fromtimestamp(1746541380, tz=timezone.utc).isoformat()
    (tmp_path / "broken.xml").write_text("<smses><sms")

    bus = MemoryBus()

    async def go():
        w = XmlWatcher(bus, tmp_path, interval_s=0.01)
        n = await w.scan_once()
        return w, n, await drain(bus, SUBJECT_RAW)

    w, n, raw = arun(go())
    assert n == 2 and w.failed_files == 1
    assert [RawSMS(**r).body for r in raw] == [body, "hello"]
    assert (tmp_path / "processed" / "sms-2025.xml").exists() and not f.exists()
    assert (tmp_path / "broken.xml").exists()  # failing file stays for the next scan


# --------------------------------------------------------------------------- DLQ worker
def _raw(body, msg_id="m1"):
    return RawSMS(msg_id=msg_id, device_id="d", sender="BANK", date="2025-05-06T00:00:00", body=body,
                  source="device")


def test_dlq_extract_raw_all_shapes():
    from smsgate_amd.services.dlq import extract_raw

    r = _raw("x").model_dump()
    assert extract_raw({"reason": "unmatched", "raw": r}) == r  # (c)
    assert extract_raw({"err": "boom", "entry": r}) == r  # (b)
    assert extract_raw({"err": "Future date", "entry": json.dumps(r)}) == r  # (a)/(d)/(e)
    assert extract_raw({"err": "x", "entry": "{not json"}) is None
    parsed = {"msg_id": "m", "amount": "1"}  # (f): writer failure — a ParsedSMS, not re-parsable
    assert extract_raw({"err": "db", "entry": json.dumps(parsed)}) is None
    assert extract_raw([1, 2]) is None


def test_dlq_reparse_routes_and_acks_everything(arun):
    from smsgate_amd.services.dlq import DlqWorker

    bus = MemoryBus()
    good = REFERENCE_CASES[0][0]

    async def go():
        await bus.publish(SUBJECT_FAILED, json.dumps({"reason": "unmatched", "raw": _raw(good).model_dump()}).encode())
        await bus.publish(SUBJECT_FAILED, json.dumps({"err": "x", "entry": _raw(good, "m2").model_dump_json()}).encode())
        await bus.publish(SUBJECT_FAILED, json.dumps({"err": "db", "entry": json.dumps({"a": 1})}).encode())
        await bus.publish(SUBJECT_FAILED, b"not json")
        w = DlqWorker(bus, ParsePipeline(RegexBackend()), reparse=True)
        await w.stage.run_until_idle()
        info = await bus.consumer_info("SMS", "parser_worker_dlq")
        return w, info, await drain(bus, SUBJECT_PARSED), await drain(bus, SUBJECT_PROCESSING)

    w, info, parsed, processing = arun(go())
    assert w.seen == 4 and w.reparsed == 2 and w.not_reparsable == 1
    assert info.num_ack_pending == 0 and info.num_pending == 0  # D16: everything acked
    assert sorted(p["msg_id"] for p in parsed) == ["m1", "m2"]
    assert len(processing) == 2


def test_dlq_reparse_failure_is_terminal(arun):
    """A message that fails every time is re-parsed exactly once: the worker
    consumes sms.failed, so a failure must not be republished there."""
    from smsgate_amd.services.dlq import DlqWorker

    bus = MemoryBus()
    calls = []

    class AlwaysFails(RegexBackend):
        async def extract_batch(self, bodies):
            calls.extend(bodies)
            return [BackendError("still broken")] * len(bodies)

    async def go():
        await bus.publish(SUBJECT_FAILED, json.dumps({"reason": "unmatched",
                                                      "raw": _raw(REFERENCE_CASES[0][0]).model_dump()}).encode())
        await bus.publish(SUBJECT_FAILED, json.dumps({"reason": "unmatched",
                                                      "raw": _raw("hello there", "m9").model_dump()}).encode())
        w = DlqWorker(bus, ParsePipeline(AlwaysFails()), reparse=True)
        await w.stage.run_until_idle(idle_s=0.3)
        info = await bus.consumer_info("SMS", "parser_worker_dlq")
        return w, info, await drain(bus, SUBJECT_PARSED), await drain(bus, SUBJECT_FAILED_FINAL)

    from prometheus_client import REGISTRY

    m0 = REGISTRY.get_sample_value("sms_dlq_reparse_failed_total") or 0.0
    w, info, parsed, final = arun(go())
    assert w.seen == 2 and w.reparsed == 2 and w.reparse_failed == 2
    assert len(calls) == 2 and len(set(calls)) == 2  # each body reached the backend exactly once
    assert info.num_pending == 0 and info.num_ack_pending == 0 and parsed == []
    # the twice-failed messages stay inspectable on the terminal subject, and are counted
    assert len(final) == 2 and all("raw" in f or "entry" in f for f in final)
    assert (REGISTRY.get_sample_value("sms_dlq_reparse_failed_total") or 0.0) - m0 == 2


def test_dlq_terminal_subject_on_reference_stream_and_rejection(arun):
    """(1) a stream created by the reference with its five subjects gains
    sms.failed.final when the DLQ worker starts (ensure_stream updates it), and a
    twice-failed message lands there; (2) if the broker refuses the terminal subject,
    the message is logged and acked -- the DLQ consumer never loops on it."""
    from smsgate_amd.bus import BusError
    from smsgate_amd.bus.base import StreamConfig
    from smsgate_amd.services.dlq import DlqWorker

    class AlwaysFails(RegexBackend):
        async def extract_batch(self, bodies):
            return [BackendError("still broken")] * len(bodies)

    env = json.dumps({"reason": "unmatched", "raw": _raw("hello there", "m9").model_dump()}).encode()
    bus = MemoryBus()

    async def go_reference_stream():
        await bus.ensure_stream(StreamConfig(name="SMS", subjects=[SUBJECT_RAW, SUBJECT_PARSED, SUBJECT_FAILED,
                                                                   "sms.processing", "sms.categorized"]))
        await bus.publish(SUBJECT_FAILED, env)
        w = DlqWorker(bus, ParsePipeline(AlwaysFails()), reparse=True)
        await w.start()
        await w.stop()
        await w.stage.run_until_idle(idle_s=0.3)
        return w, await drain(bus, SUBJECT_FAILED_FINAL)

    w, final = arun(go_reference_stream())
    assert w.reparse_failed == 1 and len(final) == 1 and w.final_rejected == 0

    class Refusing(MemoryBus):
        async def publish_many(self, items):
            if any(s == SUBJECT_FAILED_FINAL for s, _ in items):
                raise BusError("no stream captures subject 'sms.failed.final'")
            return await super().publish_many(items)

    bus2 = Refusing()

    async def go_refused():
        await bus2.publish(SUBJECT_FAILED, env)
        w = DlqWorker(bus2, ParsePipeline(AlwaysFails()), reparse=True)
        await w.stage.run_until_idle(idle_s=0.3)
        return w, await bus2.consumer_info("SMS", "parser_worker_dlq")

    w, info = arun(go_refused())
    assert w.final_rejected == 1 and w.stage.dead_lettered == 0 and w.seen == 1
    assert info.num_pending == 0 and info.num_ack_pending == 0


def test_dlq_reparse_profiler_dumps_pstats(arun, tmp_path):
    """Reparse runs inside a profiler session (dlq_worker.py:70-74); with a
    profile dir set, a cProfile dump lands there and names the parse path."""
    import pstats

    from smsgate_amd.obs.tracing import Profiler
    from smsgate_amd.services.dlq import DlqWorker

    bus = MemoryBus()
    good = REFERENCE_CASES[0][0]

    async def go():
        await bus.publish(SUBJECT_FAILED, json.dumps({"reason": "unmatched", "raw": _raw(good).model_dump()}).encode())
        w = DlqWorker(bus, ParsePipeline(RegexBackend()), reparse=True)
        w.profiler = Profiler("dlq_reparse", out_dir=str(tmp_path))
        await w.stage.run_until_idle()
        return w

    w = arun(go())
    assert w.reparsed == 1 and w.profiler.dumped is not None
    funcs = {f[2] for f in pstats.Stats(w.profiler.dumped).stats}
    assert "route_batch" in funcs
    # no dir, no SDK: a no-op session, nested use is balanced
    p = Profiler("x", out_dir="")
    with p, p:
        pass
    assert p.dumped is None and p._depth == 0


# --------------------------------------------------------------------------- notifier
def _pb_rec(i, dt, merchant="SHOP", amount="10.00", balance="100.00"):
    return {"msg_id": f"id{i}", "datetime": dt, "merchant": merchant, "amount": amount, "balance": balance,
            "currency": "AMD"}


def test_notifier_state_atomic_and_corrupt(tmp_path):
    from smsgate_amd.services.notifier import NotifierState

    p = tmp_path / "last_state.json"
    p.write_text("{corrupt")
    s = NotifierState(p)
    assert s.data["offset"] == 0 and s.last_ts < datetime.now(timezone.utc)
    s.data["offset"] = 7
    s.save()
    assert json.loads(p.read_text())["offset"] == 7
    assert [x.name for x in tmp_path.iterdir()] == ["last_state.json"]  # no temp files left


def test_notifier_cycle_sends_report_and_denies(tmp_path, arun):
    from smsgate_amd.services.notifier import CAPTION, DENY_TEXT, Notifier, NotifierState, TelegramClient
    from smsgate_amd.sinks.pocketbase import PocketBaseClient

    now = datetime.now(timezone.utc)
    pb_fake = FakePocketBase()
    pb_fake.cols["sms_data"] = [
        _pb_rec(1, (now - timedelta(days=2)).strftime("%Y-%m-%d %H:%M:%S.000Z")),
        _pb_rec(2, (now - timedelta(days=1)).strftime("%Y-%m-%d %H:%M:%S.000Z"), merchant="", balance="90.50"),
    ]
    tg_fake = FakeTelegram([{"update_id": 5, "message": {"chat": {"id": 999}, "text": "hi"}},
                            {"update_id": 6, "message": {"chat": {"id": 42}, "text": "hi"}}])

    async def go():
        pb = PocketBaseClient(base_url="http://pb", email="a@b.c", password="pw", transport=pb_fake.transport())
        tg = TelegramClient("TOKEN", transport=tg_fake.transport())
        st = NotifierState(tmp_path / "state.json")
        st.data["last_ts"] = (now - timedelta(days=3)).isoformat()
        n = Notifier(pb, tg, {42}, st, tmp_path / "out", interval_s=3600)
        sent1 = await n.run_cycle()
        sent2 = await n.run_cycle()  # nothing newer → no second report
        await n.handle_updates(await tg.get_updates(0))
        await pb.close()
        await tg.close()
        return n, st, sent1, sent2

    n, st, sent1, sent2 = arun(go())
    assert sent1 and not sent2 and n.reports_sent == 1
    reports = [s for s in tg_fake.sent if s["method"] in ("sendPhoto", "sendDocument")]
    assert reports and all(s["chat_id"] == 42 for s in reports)
    assert CAPTION in reports[0]["caption"] and "90.50 AMD" in reports[0]["caption"]
    assert (tmp_path / "out" / "payments_by_day.html").exists()
    deny = [s for s in tg_fake.sent if s["method"] == "sendMessage"]
    assert deny == [{"method": "sendMessage", "bytes": deny[0]["bytes"], "chat_id": 999,
                     "text": DENY_TEXT.format(chat_id=999)}]
    saved = json.loads((tmp_path / "state.json").read_text())
    assert saved["offset"] == 7  # both loops share one state object (R1/D13)
    assert saved["last_ts"] == st.data["last_ts"] and st.last_ts > now - timedelta(days=2)


def test_chart_totals_and_files(tmp_path):
    """The report's data and both files (dashboard/main.py:146-197 parity: daily sums per
    merchant, empty merchants as "Unknown", the newest record's balance), rendered without
    a plotting stack: inline-SVG HTML and a Pillow JPEG."""
    from datetime import date

    from smsgate_amd.services.notifier import build_chart, daily_totals
    recs = [{"amount": "100.5", "datetime": "2024-03-01 10:00:00.000Z", "merchant": "Shop A", "balance": "1 000,50",
             "currency": "AMD"},
            {"amount": "20", "datetime": "2024-03-01T12:00:00", "merchant": ""},
            {"amount": "-30", "datetime": "2024-03-02 09:00:00Z", "merchant": "Shop A"},
            {"amount": "7", "datetime": "2024-03-02 23:00:00Z", "merchant": "null", "balance": "55", "currency": "RUB"},
            {"amount": "oops", "datetime": "2024-03-02 10:00:00Z", "merchant": "bad"},
            {"amount": "5", "datetime": "not a date", "merchant": "bad"}]
    days, merchants, totals, bal = daily_totals(recs)
    assert days == [date(2024, 3, 1), date(2024, 3, 2)]
    assert merchants == ["Shop A", "Unknown"]  # by total: 70.5 vs 27
    assert totals == {(date(2024, 3, 1), "Shop A"): 100.5, (date(2024, 3, 1), "Unknown"): 20.0,
                      (date(2024, 3, 2), "Shop A"): -30.0, (date(2024, 3, 2), "Unknown"): 7.0}
    assert bal == (55.0, "RUB")
    html, img, bal2 = build_chart(recs, "Статистика", tmp_path)
    page = html.read_text(encoding="utf-8")
    assert bal2 == bal and page.count("<rect") == 4 + 2 and "Статистика" in page and "Продавец" in page
    assert img is not None and img.read_bytes()[:3] == b"\xff\xd8\xff"  # a JPEG
    with pytest.raises(ValueError):
        build_chart([{"amount": None, "datetime": None}], "t", tmp_path)


# --------------------------------------------------------------------------- MCP server
@pytest.fixture
def mcp_tools(tmp_path):
    from smsgate_amd.services.mcp_server import McpTools
    from smsgate_amd.sinks.sql import SqlSink

    return McpTools(SqlSink(f"sqlite:///{tmp_path}/mcp.sqlite"))


def _parsed(msg_id, amount="52.00", txn="debit", sender="BANK"):
    return dict(msg_id=msg_id, device_id="dev", sender=sender, date="2025-05-06T14:23:00", txn_type=txn, amount=amount,
                currency="USD", card="0018", merchant="TEST LLC", city="MOSKOW", address="",
                balance="1842.74", parser_version="llm-0.2.0", raw_body="body")


def test_mcp_tools_crud(mcp_tools, arun):
    async def go():
        t = mcp_tools
        r1 = await t.create_parsed_sms(_parsed("a"))
        r1b = await t.create_parsed_sms(_parsed("a", amount="60.00"))  # idempotent upsert by msg_id
        await t.create_parsed_sms(_parsed("b", amount="5.00", txn="credit", sender="OTHER"))
        allr = await t.find_sms_records()
        big = await t.find_sms_records(min_amount=10)
        credit = await t.find_sms_records(txn_type="credit", sender="OTHER")
        none = await t.find_sms_records(start_date="2030-01-01")
        rid = big[0]["id"]
        one = await t.get_record_by_id(rid)
        bad = await t.update_record_by_id(rid, {"merchant": "NEW", "bogus": 1})
        assert "bogus" in bad
        upd = await t.update_record_by_id(rid, {"merchant": "NEW", "amount": 61})
        after = await t.get_record_by_id(rid)
        dele = await t.delete_record_by_id(rid)
        missing = await t.get_record_by_id(rid)
        now = await t.get_current_datetime()
        return r1, r1b, allr, big, credit, none, one, upd, after, dele, missing, now

    r1, r1b, allr, big, credit, none, one, upd, after, dele, missing, now = arun(go())
    assert isinstance(r1, str) and isinstance(r1b, str)
    assert len(allr) == 2 and len(big) == 1 and Decimal(big[0]["amount"]) == Decimal("60.00")
    assert len(credit) == 1 and credit[0]["msg_id"] == "b" and none == []
    assert one["msg_id"] == "a" and after["merchant"] == "NEW"
    assert "error" in missing and isinstance(dele, str)
    datetime.fromisoformat(now)


def test_mcp_jsonrpc_http_and_sse(mcp_tools):
    from smsgate_amd.services.mcp_server import PROTOCOL_VERSION, create_mcp_app

    c = TestClient(create_mcp_app(mcp_tools))
    r = c.post("/mcp", json={"jsonrpc": "2.0", "id": 1, "method": "initialize", "params": {}}).json()
    assert r["result"]["protocolVersion"] == PROTOCOL_VERSION
    assert c.post("/mcp", json={"jsonrpc": "2.0", "method": "notifications/initialized"}).status_code == 202
    tools = c.post("/mcp", json={"jsonrpc": "2.0", "id": 2, "method": "tools/list"}).json()["result"]["tools"]
    assert {t["name"] for t in tools} == {"get_record_by_id", "find_sms_records", "update_record_by_id",
                                         "delete_record_by_id", "create_parsed_sms", "get_current_datetime"}
    call = {"jsonrpc": "2.0", "id": 3, "method": "tools/call",
            "params": {"name": "create_parsed_sms", "arguments": {"parsed_sms_data": _parsed("z")}}}
    assert c.post("/mcp", json=call).json()["result"]["isError"] is False
    call = {"jsonrpc": "2.0", "id": 4, "method": "tools/call", "params": {"name": "find_sms_records", "arguments": {}}}
    res = c.post("/mcp", json=call).json()["result"]
    assert json.loads(res["content"][0]["text"])[0]["msg_id"] == "z"
    bad = c.post("/mcp", json={"jsonrpc": "2.0", "id": 5, "method": "tools/call",
                              "params": {"name": "nope"}}).json()
    assert bad["error"]["code"] == -32602
    assert c.post("/mcp", json={"jsonrpc": "2.0", "id": 6, "method": "x"}).json()["error"]["code"] == -32601
    assert c.post("/messages/?session_id=unknown", json={}).status_code == 404


# --------------------------------------------------------------------------- Gemini REST backend
def test_gemini_http_backend_request_and_errors(monkeypatch, arun):
    from smsgate_amd.parse.backends.gemini_http import GeminiHTTPBackend
    from smsgate_amd.parse.schema import SYSTEM_INSTRUCTION

    seen = []
    flaky = {"n": 0}
    answer = {"txn_type": "debit", "date": "06.05.25 14:23", "amount": "52.00", "currency": "USD",
              "card_number": "***0018", "merchant": "TEST LLC", "city": "MOSKOW", "address": "null",
              "balance": "1842.74"}

    def handler(req: httpx.Request) -> httpx.Response:
        body = json.loads(req.content)
        seen.append((req.url.path, dict(req.url.params), body))
        text = body["contents"][0]["parts"][0]["text"]
        if text == "flaky" and flaky["n"] == 0:
            flaky["n"] += 1
            return httpx.Response(503)
        if text == "garbage":
            return httpx.Response(200, json={"candidates": [{"content": {"parts": [{"text": "no json here"}]}}]})
        if text == "denied":
            return httpx.Response(403, json={"error": "forbidden"})
        out = "```json\n" + json.dumps(answer) + "\n```"
        return httpx.Response(200, json={"candidates": [{"content": {"parts": [{"text": out}]}}]})

    async def go():
        b = GeminiHTTPBackend(api_key="K", model="gemini-x", transport=httpx.MockTransport(handler), retries=1)
        monkeypatch.setattr(asyncio, "sleep", _nosleep)
        res = await b.extract_batch(["ok", "flaky", "garbage", "denied"])
        await b.close()
        return res

    res = arun(go())
    assert res[0] == answer and res[1] == answer
    assert isinstance(res[2], BackendError) and isinstance(res[3], BackendError)
    path, params, body = seen[0]
    assert path.endswith("/models/gemini-x:generateContent") and params == {"key": "K"}
    assert body["systemInstruction"]["parts"][0]["text"] == SYSTEM_INSTRUCTION
    assert body["generationConfig"]["responseMimeType"] == "application/json"
    assert body["generationConfig"]["temperature"] == pytest.approx(0.1)


_real_sleep = asyncio.sleep


async def _nosleep(_delay, *a, **k):
    await _real_sleep(0)


def test_gemini_without_key_fails_per_message(monkeypatch, arun):
    from smsgate_amd.parse.backends.gemini_http import GeminiHTTPBackend

    monkeypatch.delenv("GEMINI_API_KEY", raising=False)
    b = GeminiHTTPBackend(api_key="", transport=httpx.MockTransport(lambda r: httpx.Response(500)))
    b.api_key = ""
    res = arun(b.extract_batch(["a"]))
    assert isinstance(res[0], BackendError)


# --------------------------------------------------------------------------- receiver
def test_receiver_store_and_list(tmp_path):
    from smsgate_amd.services.receiver import BlobStore, create_receiver_app

    c = TestClient(create_receiver_app(BlobStore(tmp_path / "hooks.sqlite")))
    r = c.post("/webhook", content=b'{"message": "hi"}')
    assert r.status_code == 201 and r.json()["status"] == "success"
    key = r.json()["key"]
    c.post("/", content=b"\xff\xfe")
    lst = c.get("/").json()
    assert lst["count"] == 2 and lst["keys"][0] == key
    assert c.get(f"/{key}").json()["body"] == '{"message": "hi"}'
    assert "body_b64" in c.get(f"/{lst['keys'][1]}").json()
    assert c.get("/nope").status_code == 404


# --------------------------------------------------------------------------- legacy tools
def test_legacy_xml_process_sync(tmp_path, arun):
    from smsgate_amd.services import legacy
    from smsgate_amd.services.xml_watcher import write_backup_xml
    from smsgate_amd.sinks.pocketbase import PocketBaseClient

    credit = "Popolnenie scheta: 100.00 AMD, karta *1234, 01.06.2025 10:00. Balans: 500.00 AMD"
    f = tmp_path / "b.xml"
    write_backup_xml(f, [("BANK", 1, REFERENCE_CASES[0][0]), ("BANK", 2, "Your OTP code: 1234"),
                         ("BANK", 3, "random text"), ("BANK", 4, credit)])
    src, pur, cre = (SqliteKV(tmp_path / n) for n in ("src.sqlite", "pur.sqlite", "cre.sqlite"))
    assert legacy.import_xml_to_cache(f, src) == 4
    st = legacy.process_cache(src, pur, cre)
    assert st["processed_debit"] >= 1 and st["skipped"] == 1 and st["failed"] >= 1
    assert legacy.process_cache(src, pur, cre)["skipped"] >= 2  # processed records are not redone
    pb_fake = FakePocketBase()

    async def go():
        async with PocketBaseClient(base_url="http://pb", email="a@b.c", password="pw",
                                    transport=pb_fake.transport()) as pb:
            a = await legacy.sync_to_pocketbase(pur, cre, pb)
            b = await legacy.sync_to_pocketbase(pur, cre, pb)
            return a, b

    a, b = arun(go())
    assert a["sms_data"] == st["processed_debit"] and b["sms_data"] == 0
    assert pb_fake.cols["sms_data"][0]["merchant"] == "TEST LLC"
    assert json.loads(legacy.dump_cache(pur))


def test_legacy_hookdeck_pagination(tmp_path, arun):
    from smsgate_amd.services import legacy

    pages = {None: {"models": [{"id": "e1", "data": {"body": {"message": REFERENCE_CASES[0][0]}}}],
                    "pagination": {"next": "c2"}},
             "c2": {"models": [{"id": "e2", "data": {"body": "plain"}}], "pagination": {}}}
    auth = []

    def handler(req):
        auth.append(req.headers["authorization"])
        return httpx.Response(200, json=pages[req.url.params.get("next")])

    cache = SqliteKV(tmp_path / "hd.sqlite")
    st = arun(legacy.fetch_hookdeck_events("KEY", "wh", cache, transport=httpx.MockTransport(handler)))
    assert st == {"events": 2, "parsed": 1} and auth == ["Bearer KEY"] * 2
    assert cache.get("e1")["parsed"]["merchant"] == "TEST LLC"


# --------------------------------------------------------------------------- PocketBase client / sink
def test_pocketbase_upsert_dedup_and_retry(arun):
    from smsgate_amd.sinks.pocketbase import PocketBaseClient, PocketBaseSink

    fake = FakePocketBase(fail_first=2)
    p = ParsedSMS(**_parsed("x1"))

    async def go():
        c = PocketBaseClient(base_url="http://pb", email="a@b.c", password="pw", transport=fake.transport(),
                             retry_min=0.001, retry_max=0.002)
        sink = PocketBaseSink(c)
        await sink.upsert_many([p])
        await sink.upsert_many([p.model_copy(update={"merchant": "CHANGED"})])
        since = await c.get_records_since("sms_data", "2000-01-01 00:00:00.000")
        await c.close()
        return since

    since = arun(go())
    recs = fake.cols["sms_data"]
    assert len(recs) == 1 and recs[0]["merchant"] == "CHANGED" and len(since) == 1
    assert any("auth-with-password" in c for c in fake.calls)


def test_pocketbase_batch_upsert_and_fallbacks(arun):
    """With the batch API, N records cost 2 x ceil(N / 50) requests (one msg_id lookup,
    one batch: PUT on msg_id-derived ids, PATCH where a msg_id is already stored under
    another id, e.g. by the reference's writer); a server without the batch API (403)
    switches the sink to per-record for good."""
    from smsgate_amd.sinks.pocketbase import PocketBaseClient, PocketBaseSink, record_id

    recs = [ParsedSMS(**_parsed(f"b{i}")) for i in range(120)]

    async def run(fake, batches):
        c = PocketBaseClient(base_url="http://pb", transport=fake.transport(), retry_min=0.001, retry_max=0.002)
        sink = PocketBaseSink(c)
        for b in batches:
            await sink.upsert_many(b)
        await c.close()
        return sink

    fake = FakePocketBase(batch_enabled=True)
    sink = arun(run(fake, [recs, [r.model_copy(update={"merchant": "NEW"}) for r in recs[:10]]]))
    stored = fake.cols["sms_data"]
    assert len(stored) == 120 and sink.batched == 130 and sink.per_record == 0
    assert sum(c == "POST /api/batch" for c in fake.calls) == 4  # 50 + 50 + 20, then 10
    assert {r["id"] for r in stored} == {record_id(f"b{i}") for i in range(120)}
    assert sum(r["merchant"] == "NEW" for r in stored) == 10

    legacy_fake = FakePocketBase(batch_enabled=True)
    legacy_fake.cols["sms_data"] = [dict(msg_id="b3", id="legacyrandomid0", merchant="OLD")]
    sink = arun(run(legacy_fake, [recs[:5]]))
    assert sink.batched == 5 and sink.per_record == 0 and sink.batch_supported is True
    assert len(legacy_fake.cols["sms_data"]) == 5  # b3 PATCHed in place, no duplicate
    assert next(r for r in legacy_fake.cols["sms_data"] if r["msg_id"] == "b3")["id"] == "legacyrandomid0"

    off = FakePocketBase(batch_enabled=False)
    sink = arun(run(off, [recs[:60], recs[60:]]))
    assert sink.batch_supported is False and sink.per_record == 120 and len(off.cols["sms_data"]) == 120
    assert sum(c == "POST /api/batch" for c in off.calls) == 1  # probed once, then per record


def test_pocketbase_paths_share_one_record_per_msg_id(arun):
    """on the reference schema (msg_id NOT unique) the batch path must not
    create a second record for a msg_id the per-record path (or the reference's
    writer) stored, and vice versa -- both paths address one record per msg_id."""
    from smsgate_amd.sinks.pocketbase import PocketBaseClient, PocketBaseSink, record_id

    fake = FakePocketBase(batch_enabled=False, unique_msg_id=False)
    fake.cols["sms_data"] = [dict(msg_id="ref0", id="referencerand01", merchant="OLD")]
    recs = [ParsedSMS(**_parsed(f"m{i}")) for i in range(6)]
    ref0 = ParsedSMS(**_parsed("ref0"))

    async def go():
        c = PocketBaseClient(base_url="http://pb", transport=fake.transport(), retry_min=0.001, retry_max=0.002)
        sink = PocketBaseSink(c)
        await sink.upsert_many(recs[:3])  # batch API off: per-record creates (derived ids)
        fake.batch_enabled = True
        sink.batch_supported = None
        # redelivery of m0..m2 + new m3..m5 + the reference's record, all through the batch path
        await sink.upsert_many([r.model_copy(update={"merchant": "B"}) for r in recs] + [ref0])
        fake.batch_enabled = False
        sink.batch_supported = False
        await sink.upsert_many([recs[4].model_copy(update={"merchant": "P"})])  # per-record after batch
        await c.close()
        return sink

    sink = arun(go())
    stored = fake.cols["sms_data"]
    by_msg = {}
    for r in stored:
        by_msg.setdefault(r["msg_id"], []).append(r)
    assert all(len(v) == 1 for v in by_msg.values()), {k: len(v) for k, v in by_msg.items()}
    assert len(stored) == 7 and sink.batched == 7
    assert by_msg["ref0"][0]["id"] == "referencerand01" and by_msg["ref0"][0]["merchant"] == "TEST LLC"
    assert all(by_msg[f"m{i}"][0]["id"] == record_id(f"m{i}") for i in range(6))
    assert by_msg["m4"][0]["merchant"] == "P" and by_msg["m0"][0]["merchant"] == "B"


# --------------------------------------------------------------------------- CLI
def test_cli_parses_every_service():
    from smsgate_amd.cli import build_parser

    p = build_parser()
    for argv in (["gateway"], ["parser", "--group", "g", "--backend", "regex"], ["writer"], ["dlq", "--reparse"],
                 ["xml-watcher"], ["notifier"], ["mcp-server"], ["receiver"], ["bus-server", "--listen", "unix:///x"],
                 ["engine-server", "--max-slots", "64"], ["pipeline"], ["db", "upgrade"], ["legacy", "import-xml"],
                 ["config"]):
        assert p.parse_args(argv).cmd == argv[0]


def test_cli_db_roundtrip(tmp_path, capsys):
    from smsgate_amd.cli import main

    url = f"sqlite:///{tmp_path}/c.sqlite"
    assert main(["db", "upgrade", "--url", url]) == 0
    main(["db", "current", "--url", url])
    main(["db", "downgrade", "base", "--url", url])
    main(["db", "current", "--url", url])
    out = capsys.readouterr().out.split()
    assert "0002_sms_indexes" in out[-2] or "0002_sms_indexes" in out


# --------------------------------------------------------------------------- ngrok tunnel
def test_tunnel_disabled_sdk_and_missing(monkeypatch):
    import sys
    import types

    from smsgate_amd.config import Settings
    from smsgate_amd.services import tunnel

    assert tunnel.open_tunnel(Settings.load({}, env_file=None), 9001) is None
    calls = []

    class _Listener:
        def url(self):
            return "https://x.ngrok.app"

    fake = types.ModuleType("ngrok")
    fake.forward = lambda port, **kw: (calls.append((port, kw)), _Listener())[1]
    fake.disconnect = lambda url: calls.append(("disconnect", url))
    monkeypatch.setitem(sys.modules, "ngrok", fake)
    s = Settings.load({"ENABLE_NGROK": "true", "NGROK_AUTHTOKEN": "tok", "NGROK_DOMAIN": "d.ngrok.app"},
                      env_file=None)
    t = tunnel.open_tunnel(s, 9001)
    assert t.url == "https://x.ngrok.app"
    assert calls[0] == (9001, {"authtoken": "tok", "domain": "d.ngrok.app"})
    t.close()
    assert calls[-1] == ("disconnect", "https://x.ngrok.app")
    monkeypatch.delitem(sys.modules, "ngrok")
    monkeypatch.setattr(tunnel.shutil, "which", lambda name: None)
    monkeypatch.setitem(sys.modules, "ngrok", None)  # import ngrok -> ImportError
    assert tunnel.open_tunnel(s, 9001) is None


def test_engine_metrics_exporter():
    """The engine-server's Prometheus exporter turns engine counters into metrics."""
    from types import SimpleNamespace

    from smsgate_amd.obs import metrics as M
    from smsgate_amd.serving.engine import EngineStats

    eng = SimpleNamespace(stats=EngineStats(), active={1: "a", 2: "b"}, waiting=[1, 2, 3])
    ex = M.EngineMetricsExporter(eng)

    def val(name, **labels):
        return M.REGISTRY.get_sample_value(name, labels) or 0.0

    before = (val("llm_tokens_total", phase="decode"), val("llm_sequences_completed_total"))
    eng.stats.decode_steps, eng.stats.decode_row_steps, eng.stats.completed = 4, 1000, 17
    eng.stats.prefill_tokens, eng.stats.steps, eng.stats.step_s = 500, 2, 0.01
    ex.export_once()
    assert val("llm_tokens_total", phase="decode") - before[0] == 1000
    assert val("llm_sequences_completed_total") - before[1] == 17
    assert val("llm_active_sequences") == 2 and val("llm_waiting_sequences") == 3
    ex.export_once()  # no new work: counters unchanged
    assert val("llm_tokens_total", phase="decode") - before[0] == 1000


def test_engine_server_refuses_random_weights(tmp_path, monkeypatch):
    """No LLM_CHECKPOINT / --checkpoint and no bundled 135M weights: engine-server
    exits non-zero before touching a GPU instead of serving random init
    (ADVICE cli.py:190)."""
    import subprocess
    import sys

    env = {k: v for k, v in __import__("os").environ.items() if k != "LLM_CHECKPOINT"}
    cmd = [sys.executable, "-m", "smsgate_amd", "engine-server", "--listen", f"unix://{tmp_path}/e.sock"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no trained checkpoint" in r.stderr
    env["LLM_CHECKPOINT"] = str(tmp_path / "missing.safetensors")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "does not exist" in r.stderr

    from smsgate_amd.parse.backends.local_llm import MissingCheckpoint, resolve_checkpoint

    monkeypatch.delenv("LLM_CHECKPOINT", raising=False)
    with pytest.raises(MissingCheckpoint):
        resolve_checkpoint("smollm-135m")
    assert resolve_checkpoint("smollm-135m", random_init=True) is None
    assert resolve_checkpoint("small").endswith("extractor-small.safetensors")  # bundled


def test_observe_many_equals_repeated_observe():
    """One latency per message, recorded in O(1) per batch: the exported samples equal
    n observe() calls (the reference times every message, worker.py:130-133)."""
    from prometheus_client import CollectorRegistry, Histogram, Summary

    from smsgate_amd.obs.metrics import observe_many

    reg = CollectorRegistry()
    h1, h2 = (Histogram(f"h{i}_seconds", "x", registry=reg, buckets=(0.001, 0.01, 0.1, 1)) for i in (1, 2))
    s1, s2 = (Summary(f"s{i}_seconds", "x", registry=reg) for i in (1, 2))
    for v, n in ((0.005, 7), (0.1, 3), (5.0, 2), (0.0001, 4), (0.01, 1)):
        for _ in range(n):
            h1.observe(v)
            s1.observe(v)
        observe_many(h2, v, n)
        observe_many(s2, v, n)

    def samples(m):
        return [(x.name.split("_", 1)[1], x.labels, round(x.value, 9)) for x in m.collect()[0].samples
                if not x.name.endswith("created")]

    assert samples(h1) == samples(h2) and samples(s1) == samples(s2)
