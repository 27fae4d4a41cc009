"""NATS wire-protocol compatibility: NatsBus client <-> NATS front-end broker.

Every test runs against both front-ends: the Python one (``NatsFrontend`` on the
in-process engine) and the C++ one (``smsgate-busd --nats-listen``).
Both sides are ours (nats-py and nats-server are not on the image), so the raw
protocol tests below also drive the front-end with hand-written frames the way
the reference's nats-py services would (push durable consumer, ``$JS.ACK``
replies) — parity with a real nats-server beyond these frames is unpinned.
"""
from __future__ import annotations

import asyncio
import json

import pytest

from conftest import REFERENCE_CASES
from smsgate_amd.bus import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_RAW, MemoryBus, connect
from smsgate_amd.bus import nats_proto as P
from smsgate_amd.bus.base import BusError
from smsgate_amd.bus.nats_client import NatsBus
from smsgate_amd.bus.nats_server import NatsFrontend
from smsgate_amd.native import BUSD, available, spawn_busd


class _Busd:
    """smsgate-busd with only a NATS listener, shaped like NatsFrontend (async close)."""

    def __init__(self) -> None:
        self.broker = spawn_busd([], None, nats_listen="tcp://127.0.0.1:0")
        self.port = self.broker.nats_port

    async def close(self) -> None:
        self.broker.stop()


@pytest.fixture(params=["python", "busd"])
def kind(request):
    if request.param == "busd" and not available(BUSD):
        pytest.skip("smsgate-busd not built")
    return request.param


async def _start(kind="python"):
    if kind == "busd":
        fe = _Busd()
        return None, fe, fe.port
    broker = MemoryBus()
    fe = NatsFrontend(broker)
    port = await fe.start("127.0.0.1", 0)
    return broker, fe, port


def test_publish_fetch_ack_nak_term(arun, kind):
    async def go():
        broker, fe, port = await _start(kind)
        nb = await connect(f"nats://127.0.0.1:{port}")
        assert isinstance(nb, NatsBus) and await nb.ping()
        si = await nb.ensure_stream()
        assert si.config.name == "SMS" and SUBJECT_RAW in si.config.subjects
        acks = await nb.publish_many([(SUBJECT_RAW, b"a"), (SUBJECT_RAW, b"b"), (SUBJECT_RAW, b"c")])
        assert [a.seq for a in acks] == [1, 2, 3] and acks[0].stream == "SMS"
        sub = await nb.subscribe(SUBJECT_RAW, "w1", ack_wait=0.3)
        got = await sub.fetch(10, 1.0)
        assert [m.data for m in got] == [b"a", b"b", b"c"]
        assert got[0].metadata.stream == "SMS" and got[0].metadata.consumer == "w1"
        await got[0].ack()
        await got[1].nak()
        await got[2].term()
        await asyncio.sleep(0.05)
        again = await sub.fetch(10, 1.0)
        assert [m.data for m in again] == [b"b"] and again[0].metadata.num_delivered == 2
        await again[0].ack()
        await asyncio.sleep(0.05)
        info = await nb.consumer_info("SMS", "w1")
        assert info.num_ack_pending == 0 and info.num_pending == 0
        assert await sub.fetch(5, 0.1) == []  # 408 / empty
        st = await nb.stream_info("SMS")
        assert st.last_seq == 3
        # unacked deliveries come back after ack_wait
        await nb.publish(SUBJECT_RAW, b"d")
        first = await sub.fetch(1, 1.0)
        assert first[0].data == b"d"
        redeliv = await sub.fetch(1, 2.0)
        assert redeliv and redeliv[0].data == b"d" and redeliv[0].metadata.num_delivered == 2
        await redeliv[0].ack()
        await nb.close()
        await fe.close()

    arun(go())


def test_competing_consumers_share_a_durable(arun, kind):
    async def go():
        broker, fe, port = await _start(kind)
        a = await connect(f"nats://127.0.0.1:{port}")
        b = await connect(f"nats://127.0.0.1:{port}")
        await a.publish_many([(SUBJECT_PARSED, str(i).encode()) for i in range(40)])
        sa = await a.subscribe(SUBJECT_PARSED, "pb_writer")
        sb = await b.subscribe(SUBJECT_PARSED, "pb_writer")
        seen = []
        for _ in range(10):
            for s in (sa, sb):
                for m in await s.fetch(3, 0.2):
                    seen.append(int(m.data))
                    await m.ack()
        assert sorted(seen) == list(range(40))  # each message once across both processes
        await a.close()
        await b.close()
        await fe.close()

    arun(go())


def test_publish_to_uncaptured_subject_and_errors(arun, kind):
    async def go():
        broker, fe, port = await _start(kind)
        nb = await connect(f"nats://127.0.0.1:{port}")
        with pytest.raises(BusError):
            await nb.publish("not.a.stream", b"x")
        with pytest.raises(BusError):
            await nb.consumer_info("SMS", "missing")
        with pytest.raises(BusError):
            await nb.stream_info("NOPE")
        await nb.close()
        await fe.close()

    arun(go())


async def _raw(port):
    r, w = await asyncio.open_connection("127.0.0.1", port)
    info = await P.read_frame(r)
    assert info.op == "INFO" and json.loads(info.args[0])["jetstream"] is True
    w.write(b'CONNECT {"verbose":false,"headers":true}\r\nPING\r\n')
    assert (await P.read_frame(r)).op == "PONG"
    return r, w


def test_raw_protocol_push_consumer_like_nats_py(arun, kind):
    """What nats-py's ``js.subscribe(subject, durable=...)`` + ``msg.ack()`` sends."""

    async def go():
        broker, fe, port = await _start(kind)
        r, w = await _raw(port)
        w.write(b"SUB _INBOX.me.* 1\r\n")
        # stream lookup by subject, then a push durable on a deliver inbox
        w.write(P.pub_bytes("$JS.API.STREAM.NAMES", P.dumps({"subject": SUBJECT_FAILED}), "_INBOX.me.1"))
        f = await P.read_frame(r)
        assert json.loads(f.payload)["streams"] == ["SMS"]
        cfg = {"stream_name": "SMS", "config": {"durable_name": "parser_worker_dlq", "deliver_subject": "_INBOX.dlv",
                                                "ack_policy": "explicit", "filter_subject": SUBJECT_FAILED}}
        w.write(b"SUB _INBOX.dlv 2\r\n")
        w.write(P.pub_bytes("$JS.API.CONSUMER.CREATE.SMS", P.dumps(cfg), "_INBOX.me.2"))
        f = await P.read_frame(r)
        assert json.loads(f.payload)["name"] == "parser_worker_dlq"
        # js.publish = PUB with a reply inbox -> PubAck
        w.write(P.pub_bytes(SUBJECT_FAILED, b'{"err":"x"}', "_INBOX.me.3"))
        frames = [await asyncio.wait_for(P.read_frame(r), 2.0) for _ in range(2)]
        by_sid = {fr.args[1]: fr for fr in frames}
        assert json.loads(by_sid["1"].payload) == {"stream": "SMS", "seq": 1}
        dlv = by_sid["2"]
        assert dlv.payload == b'{"err":"x"}' and dlv.args[2].startswith("$JS.ACK.SMS.parser_worker_dlq.1.1.")
        w.write(P.pub_bytes(dlv.args[2], b"+ACK"))
        await w.drain()
        await asyncio.sleep(0.05)
        nb = await connect(f"nats://127.0.0.1:{port}")
        ci = await nb.consumer_info("SMS", "parser_worker_dlq")
        assert ci.num_ack_pending == 0 and ci.ack_floor == 1
        await nb.close()
        # core request/reply between two plain clients
        r2, w2 = await _raw(port)
        w2.write(b"SUB svc.echo 7\r\n")
        await w2.drain()
        await asyncio.sleep(0.05)
        w.write(P.pub_bytes("svc.echo", b"ping", "_INBOX.me.9"))
        req = await P.read_frame(r2)
        w2.write(P.pub_bytes(req.args[2], b"pong"))
        await w2.drain()
        resp = await asyncio.wait_for(P.read_frame(r), 2.0)
        assert resp.payload == b"pong"
        w.close()
        w2.close()
        await fe.close()

    arun(go())


def test_parser_stage_over_nats(arun, kind):
    """The unchanged parser stage running on the nats:// bus."""
    from smsgate_amd.models import RawSMS
    from smsgate_amd.parse import ParsePipeline
    from smsgate_amd.parse.backends import RegexBackend
    from smsgate_amd.services.parser import ParserWorker

    async def go():
        broker, fe, port = await _start(kind)
        nb = await connect(f"nats://127.0.0.1:{port}")
        body = REFERENCE_CASES[0][0]
        raw = RawSMS(msg_id="n1", device_id="d", sender="BANK", date="2025-05-06T00:00:00", body=body, source="device")
        await nb.publish(SUBJECT_RAW, raw.model_dump_json().encode())
        w = ParserWorker(nb, ParsePipeline(RegexBackend()), stats_interval=0)
        await w.stage.run_until_idle()
        sub = await nb.subscribe(SUBJECT_PARSED, "check")
        got = await sub.fetch(5, 1.0)
        assert len(got) == 1 and json.loads(got[0].data)["merchant"] == "TEST LLC"
        assert w.counts["ok"] == 1
        await nb.close()
        await fe.close()

    arun(go())


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_broker_process_crash_recovery_over_nats(tmp_path, arun, kind):
    """bus-server subprocess (journaled; ``--native`` = smsgate-busd) + NATS clients:
    kill -9 mid-stream, restart, unacked and unread messages are still there."""
    import os
    import signal
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nport, mport = _free_port(), _free_port()

    def start():
        return subprocess.Popen([sys.executable, "-m", "smsgate_amd", "bus-server", "--listen",
                                 f"tcp://127.0.0.1:{mport}", "--nats-listen", f"tcp://127.0.0.1:{nport}",
                                 "--data", str(tmp_path / "bus")] + (["--native"] if kind == "busd" else []),
                                cwd=root,
                                stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)

    async def connect_retry():
        for _ in range(100):
            try:
                return await connect(f"nats://127.0.0.1:{nport}")
            except (OSError, BusError, asyncio.TimeoutError):
                await asyncio.sleep(0.1)
        raise RuntimeError("broker did not come up")

    proc = start()
    try:
        async def phase1():
            nb = await connect_retry()
            await nb.ensure_stream()
            await nb.publish_many([(SUBJECT_RAW, f"m{i}".encode()) for i in range(10)])
            sub = await nb.subscribe(SUBJECT_RAW, "pw", ack_wait=1.0)
            got = await sub.fetch(4, 2.0)
            for m in got[:2]:
                await m.ack()  # m0, m1 acked; m2, m3 delivered but unacked
            await asyncio.sleep(0.2)
            await nb.close()
            return [m.data for m in got]

        first = arun(phase1())
        assert first == [b"m0", b"m1", b"m2", b"m3"]
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait(10)
        proc = start()

        async def phase2():
            nb = await connect_retry()
            sub = await nb.subscribe(SUBJECT_RAW, "pw", ack_wait=1.0)
            seen = []
            t_end = time.monotonic() + 10
            while len(seen) < 8 and time.monotonic() < t_end:
                for m in await sub.fetch(10, 1.0):
                    seen.append(m.data)
                    await m.ack()
            await nb.close()
            return seen

        rest = arun(phase2())
        assert sorted(rest) == sorted(f"m{i}".encode() for i in range(2, 10))
    finally:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        proc.wait(10)


def test_queue_groups_headers_and_no_wait_status(arun, kind):
    """Core queue groups share a subject's messages; headers survive JetStream capture
    and come back on delivery; a partially filled no_wait pull ends with a 404 status."""

    async def go():
        broker, fe, port = await _start(kind)
        r1, w1 = await _raw(port)
        r2, w2 = await _raw(port)
        for w in (w1, w2):
            w.write(b"SUB jobs.* workers 1\r\nPING\r\n")
        for r in (r1, r2):
            assert (await P.read_frame(r)).op == "PONG"
        pub, wp = await _raw(port)
        for i in range(20):
            wp.write(P.pub_bytes(f"jobs.{i}", str(i).encode()))
        wp.write(b"PING\r\n")
        await wp.drain()
        assert (await P.read_frame(pub)).op == "PONG"
        got = []
        for r in (r1, r2):
            while True:
                try:
                    f = await asyncio.wait_for(P.read_frame(r), 0.3)
                except asyncio.TimeoutError:
                    break
                got.append(int(f.payload))
        assert sorted(got) == list(range(20))  # each message to exactly one group member
        nb = await connect(f"nats://127.0.0.1:{port}")
        await nb.publish(SUBJECT_RAW, b"with-headers", headers={"Nats-Msg-Id": "m-1", "X-Trace": "abc"})
        await nb.publish(SUBJECT_RAW, b"plain")
        sub = await nb.subscribe(SUBJECT_RAW, "hdr")
        t0 = asyncio.get_running_loop().time()
        msgs = await sub.fetch(10, 1.0)  # 2 available: the no_wait pull must end at once (404)
        assert asyncio.get_running_loop().time() - t0 < 0.5
        assert [m.data for m in msgs] == [b"with-headers", b"plain"]
        assert msgs[0].headers == {"Nats-Msg-Id": "m-1", "X-Trace": "abc"} and not msgs[1].headers
        for m in msgs:
            await m.ack()
        await nb.close()
        for w in (w1, w2, wp):
            w.close()
        await fe.close()

    arun(go())
