"""HTTP gateway contract (reference tests/api_gateway/test_main.py, re-designed:
the bus is injected instead of patching a module-global NATS singleton)."""
import json

import pytest
from fastapi.testclient import TestClient

from smsgate_amd.bus import MemoryBus, SUBJECT_RAW
from smsgate_amd.models import RawSMS, get_md5_hash
from smsgate_amd.obs import clear_errors, recent_errors
from smsgate_amd.services.gateway import create_app


class _DownBus(MemoryBus):
    async def ping(self) -> bool:
        raise ConnectionError("bus down")

    async def publish(self, *a, **k):
        raise ConnectionError("bus down")

    async def publish_many(self, *a, **k):
        raise ConnectionError("bus down")


@pytest.fixture
def bus():
    return MemoryBus()


@pytest.fixture
def client(bus):
    async def get_bus():
        return bus

    with TestClient(create_app(get_bus)) as c:
        yield c


@pytest.fixture
def valid_payload():
    return {
        "device_id": "android-pixel-8a",
        "msg_id": "1718291822123",  # extra key, ignored like in the reference
        "message": "APPROVED PURCHASE DB SALE: …",
        "sender": "AMTBBANK",
        "timestamp": 1749808562,
        "source": "device",
    }


def test_health_ok(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.json() == {"status": "ok"}


def test_health_bus_down():
    bus = _DownBus()

    async def get_bus():
        return bus

    clear_errors()
    with TestClient(create_app(get_bus, ensure_stream_on_start=False)) as c:
        r = c.get("/health")
    assert r.status_code == 503 and r.json() == {"status": "redis_down"}
    assert recent_errors()  # captured, like sentry_capture in the reference test


def test_post_sms_raw_publishes_exact_bytes(client, bus, valid_payload, arun):
    r = client.post("/sms/raw", json=valid_payload)
    assert r.status_code == 202 and r.json() == {"result": "queued"}
    expected = RawSMS(
        msg_id=get_md5_hash(valid_payload["message"]),
        sender=valid_payload["sender"],
        body=valid_payload["message"],
        date=str(valid_payload["timestamp"]),
        device_id=valid_payload["device_id"],
        source=valid_payload["source"],
    ).model_dump_json().encode("utf-8")

    async def read():
        sub = await bus.subscribe(SUBJECT_RAW, "t")
        return await sub.fetch(10, 0.1)

    msgs = arun(read())
    assert len(msgs) == 1 and msgs[0].data == expected
    assert msgs[0].subject == SUBJECT_RAW


def test_post_missing_source_is_400(client, valid_payload):
    # Quirk kept: the DTO default None fails RawSMS's Literal.
    valid_payload.pop("source")
    r = client.post("/sms/raw", json=valid_payload)
    assert r.status_code == 400 and r.json() == {"detail": "Invalid payload"}


def test_post_empty_sender_is_400(client, valid_payload):
    valid_payload["sender"] = ""
    assert client.post("/sms/raw", json=valid_payload).status_code == 400


def test_post_schema_mismatch_is_422(client, valid_payload):
    valid_payload["timestamp"] = "not-an-int"
    assert client.post("/sms/raw", json=valid_payload).status_code == 422


def test_post_publish_failure_is_500(valid_payload):
    bus = _DownBus()

    async def get_bus():
        return bus

    with TestClient(create_app(get_bus, ensure_stream_on_start=False)) as c:
        r = c.post("/sms/raw", json=valid_payload)
    assert r.status_code == 500 and r.json() == {"detail": "Internal error"}


def test_batch_and_metrics(client, bus, valid_payload, arun):
    items = []
    for i in range(3):
        p = dict(valid_payload)
        p["message"] = f"msg {i}"
        items.append(p)
    r = client.post("/sms/raw/batch", json=items)
    assert r.status_code == 202 and r.json()["count"] == 3
    m = client.get("/metrics")
    assert m.status_code == 200 and b"api_gateway_requests_total" in m.content

    async def read():
        sub = await bus.subscribe(SUBJECT_RAW, "t2")
        return await sub.fetch(10, 0.1)

    got = arun(read())
    assert [json.loads(x.data)["body"] for x in got] == ["msg 0", "msg 1", "msg 2"]


def test_concurrent_posts_share_round_trips(bus, valid_payload, arun):
    """Concurrent POST /sms/raw requests are coalesced into publish_many round trips;
    every request still gets its own 202 only after its message is on the bus."""
    import asyncio

    import httpx

    async def get_bus():
        return bus

    app = create_app(get_bus, ensure_stream_on_start=False)

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://gw") as c:
            async def one(i):
                p = dict(valid_payload)
                p["message"] = f"concurrent {i}"
                return await c.post("/sms/raw", json=p)

            rs = await asyncio.gather(*(one(i) for i in range(200)))
        sub = await bus.subscribe(SUBJECT_RAW, "check")
        got = await sub.fetch(500, 0.1)
        return rs, got

    rs, got = arun(go())
    assert all(r.status_code == 202 and r.json() == {"result": "queued"} for r in rs)
    assert sorted(json.loads(m.data)["body"] for m in got) == sorted(f"concurrent {i}" for i in range(200))
    (co,) = app.state.coalescers.values()
    assert co.published == 200 and co.round_trips < 200
