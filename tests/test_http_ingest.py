"""Native HTTP ingestion (smsgate-busd ``--http-listen``, csrc/http_ingest.hpp) is a
differential copy of the Python gateway's contract (services/gateway.py, which
mirrors services/api_gateway/main.py:106-134): for every payload both answer the
same status, and every accepted SMS lands on ``sms.raw`` as the same bytes
(``RawSMS.model_dump_json()``, msg_id = md5(message))."""
import json
import socket

import pytest
from fastapi.testclient import TestClient

from conftest import REFERENCE_CASES
from smsgate_amd.bus import SUBJECT_RAW, MemoryBus
from smsgate_amd.native import BUSD, available, spawn_busd
from smsgate_amd.services.gateway import create_app

pytestmark = pytest.mark.skipif(not available(BUSD), reason="native broker not built")

BASE = {"device_id": "android-pixel-8a", "message": REFERENCE_CASES[0][0], "sender": "AMTBBANK",
        "timestamp": 1749808562, "source": "device"}


def _case(**kw):
    d = dict(BASE)
    for k, v in kw.items():
        if v is _DROP:
            d.pop(k)
        else:
            d[k] = v
    return d


_DROP = object()
CASES = [
    _case(),
    _case(source="xml"),
    _case(message="Оплата 1 500,00 ₽ — кафе «Ромашка» 😀"),  # non-ASCII kept as UTF-8
    _case(message='quote " backslash \\ ctl \x01\x1f\b\f\n\r\t del \x7f slash /'),
    _case(msg_id="extra keys are ignored"),
    _case(timestamp="1749808562"),
    _case(timestamp=" +12 "),
    _case(timestamp="1_000"),
    _case(timestamp="12.000"),
    _case(timestamp=1749808562.0),
    _case(timestamp=True),
    _case(timestamp=-5),
    _case(timestamp=12.5),          # 422 int_from_float
    _case(timestamp="12.5"),        # 422
    _case(timestamp="0x10"),        # 422
    _case(timestamp="1__0"),        # 422
    _case(timestamp=None),          # 422
    _case(timestamp=_DROP),         # 422 missing
    _case(device_id=7),             # 422 string_type
    _case(message=_DROP),           # 422
    _case(source=_DROP),            # 400: RawSMS(source=None) (a kept quirk)
    _case(source=None),             # 400
    _case(source="web"),            # 400
    _case(source=3),                # 422
    _case(message=""),              # 400: body min_length 1
    _case(sender=""),               # 400
    [1, 2],                         # 422: not an object
]


@pytest.fixture(scope="module")
def busd(tmp_path_factory):
    d = tmp_path_factory.mktemp("httpbus")
    b = spawn_busd(f"unix://{d}/bus.sock", str(d / "data"), http_listen="tcp://127.0.0.1:0")
    yield b
    b.stop()


def _http(port, method, path, body=None, extra_headers="", raw=None):
    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    data = b"" if body is None else (body if isinstance(body, bytes) else json.dumps(body).encode())
    req = raw or (f"{method} {path} HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
                  f"Content-Length: {len(data)}\r\nConnection: close\r\n{extra_headers}\r\n").encode() + data
    s.sendall(req)
    buf = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        buf += chunk
    s.close()
    return buf


def _parse_responses(buf):
    out = []
    while buf:
        head, rest = buf.split(b"\r\n\r\n", 1)
        status = int(head.split(b" ", 2)[1])
        clen = next(int(line.split(b":")[1]) for line in head.split(b"\r\n") if line.lower().startswith(b"content-length"))
        out.append((status, rest[:clen]))
        buf = rest[clen:]
    return out


async def _drain_raw(bus, durable):
    sub = await bus.subscribe(SUBJECT_RAW, durable)
    got = []
    while True:
        ms = await sub.fetch(500, 0.2)
        if not ms:
            return got
        for m in ms:
            got.append(bytes(m.data))
            await m.ack()


def test_same_status_and_bytes_as_python_gateway(busd, arun):
    from smsgate_amd.bus import connect

    pybus = MemoryBus()

    async def get_bus():
        return pybus

    statuses = []
    with TestClient(create_app(get_bus, ensure_stream_on_start=False)) as c:
        for case in CASES:
            py = c.post("/sms/raw", json=case)
            (st, body), = _parse_responses(_http(busd.http_port, "POST", "/sms/raw", case))
            statuses.append(st)
            assert st == py.status_code, (case, st, py.status_code, body)
            if st in (202, 400):
                assert json.loads(body) == py.json(), case
            elif st == 422:  # same error types and locations as FastAPI / pydantic
                ours = [(e["type"], e["loc"]) for e in json.loads(body)["detail"]]
                theirs = [(e["type"], e["loc"]) for e in py.json()["detail"]]
                assert ours == theirs, (case, ours, theirs)

    async def go():
        nb = await connect(f"unix://{busd.listens[0][7:]}", shared=False)
        try:
            return await _drain_raw(nb, "diff"), await _drain_raw(pybus, "diff")
        finally:
            await nb.close()

    native, python = arun(go())
    assert native == python and len(native) == statuses.count(202) >= 12


def test_batch_health_metrics_and_errors(busd, arun):
    ok = [_case(message=f"batch {i}") for i in range(5)]
    (st, body), = _parse_responses(_http(busd.http_port, "POST", "/sms/raw/batch", ok))
    assert st == 202 and json.loads(body) == {"result": "queued", "count": 5}
    # one bad item: 400 and NOTHING of the batch is stored
    (st, body), = _parse_responses(_http(busd.http_port, "POST", "/sms/raw/batch", ok[:2] + [_case(source="web")]))
    assert st == 400 and json.loads(body) == {"detail": "Invalid payload"}
    (st, _), = _parse_responses(_http(busd.http_port, "POST", "/sms/raw/batch", BASE))
    assert st == 422
    (st, body), = _parse_responses(_http(busd.http_port, "GET", "/health"))
    assert st == 200 and json.loads(body) == {"status": "ok"}
    (st, _), = _parse_responses(_http(busd.http_port, "GET", "/sms/raw"))
    assert st == 405
    (st, _), = _parse_responses(_http(busd.http_port, "GET", "/nope"))
    assert st == 404
    (st, body), = _parse_responses(_http(busd.http_port, "GET", "/metrics"))
    assert st == 200 and b'api_gateway_requests_total{endpoint="/sms/raw/batch",status="202"}' in body
    (st, _), = _parse_responses(_http(busd.http_port, "POST", "/sms/raw", b"{not json"))
    assert st == 422


def test_keep_alive_pipelining(busd):
    """Three requests in one write on one connection: three answers, in order."""
    reqs = b""
    for i, case in enumerate([_case(message="p1"), _case(source="web"), _case(message="p3")]):
        data = json.dumps(case).encode()
        close = "Connection: close\r\n" if i == 2 else ""
        reqs += (f"POST /sms/raw HTTP/1.1\r\nHost: t\r\nContent-Length: {len(data)}\r\n{close}\r\n").encode() + data
    got = _parse_responses(_http(busd.http_port, None, None, raw=reqs))
    assert [s for s, _ in got] == [202, 400, 202]
