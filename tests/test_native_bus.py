"""Native C++ broker (smsgate-busd) vs the Python broker: protocol, semantics, journal compatibility.

The Python engine (smsgate_amd/bus/engine.py) is the specification: a seeded
random workload is replayed against both brokers through the same RemoteBus
client and every observable result must be identical.
"""
import asyncio
import random

import pytest

from smsgate_amd import native
from smsgate_amd.bus import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_RAW, connect
from smsgate_amd.bus.filelog import FileLog, open_file_bus
from smsgate_amd.bus.server import serve


@pytest.fixture(scope="module", autouse=True)
def _built():
    from smsgate_amd.native import build

    build.build()
    assert native.available()


def test_roundtrip_and_long_poll(tmp_path, arun):
    sock = f"unix://{tmp_path}/busd.sock"

    async def go():
        srv = await serve(sock, str(tmp_path / "data"), native=True)
        c1 = await connect(sock, shared=False)
        c2 = await connect(sock, shared=False)
        assert await c1.ping()
        await c1.ensure_stream()
        acks = await c1.publish_many([(SUBJECT_RAW, b"a"), (SUBJECT_RAW, b"b"), (SUBJECT_PARSED, b"p")])
        assert [(a.stream, a.seq) for a in acks] == [("SMS", 1), ("SMS", 2), ("SMS", 3)]
        s1 = await c1.subscribe(SUBJECT_RAW, "grp")
        s2 = await c2.subscribe(SUBJECT_RAW, "grp")
        m1 = await s1.fetch(1, 0.5)
        m2 = await s2.fetch(1, 0.5)
        assert sorted(x.data for x in m1 + m2) == [b"a", b"b"]
        for m in m1 + m2:
            await m.ack()
        await asyncio.sleep(0.05)
        info = await c2.consumer_info("SMS", "grp")
        assert info.num_ack_pending == 0 and info.num_pending == 0
        si = await c1.stream_info("SMS")
        assert si.messages == 3 and si.last_seq == 3
        waiter = asyncio.create_task(s1.fetch(1, 5.0))
        await asyncio.sleep(0.05)
        await c2.publish(SUBJECT_RAW, b"late", {"h": "v"})
        got = await waiter
        assert [m.data for m in got] == [b"late"] and got[0].headers == {"h": "v"}
        # timeout with nothing to deliver
        assert await s2.fetch(4, 0.05) == []
        # errors come back as BusError, the connection survives
        with pytest.raises(Exception, match="not found"):
            await c1.consumer_info("SMS", "nope")
        assert await c1.ping()
        await c1.close()
        await c2.close()
        await srv.close()

    arun(go())


def test_ack_wait_redelivery_and_max_deliver(tmp_path, arun):
    sock = f"unix://{tmp_path}/busd.sock"

    async def go():
        srv = await serve(sock, None, native=True)
        c = await connect(sock, shared=False)
        await c.publish(SUBJECT_RAW, b"x")
        sub = await c.subscribe(SUBJECT_RAW, "w", ack_wait=0.2, max_deliver=2)
        a = await sub.fetch(1, 0.5)
        assert a[0].metadata.num_delivered == 1
        b = await sub.fetch(1, 2.0)  # long-poll wakes at the redelivery deadline
        assert b[0].data == b"x" and b[0].metadata.num_delivered == 2
        assert await sub.fetch(1, 0.5) == []  # max_deliver reached: dropped
        await c.close()
        await srv.close()

    arun(go())


async def _workload(c, seed, n_ops=400, prefix="d"):
    """A deterministic op sequence; returns every observable result (timestamps dropped)."""
    rng = random.Random(seed)
    subjects = [SUBJECT_RAW, SUBJECT_PARSED, SUBJECT_FAILED]
    out = []
    subs = {}
    held = {}
    await c.ensure_stream()
    for _ in range(n_ops):
        op = rng.random()
        if op < 0.3:
            acks = await c.publish_many([(rng.choice(subjects), rng.randbytes(rng.randint(0, 40)))
                                         for _ in range(rng.randint(1, 6))])
            out.append(("pub", [(a.stream, a.seq) for a in acks]))
        elif op < 0.4 or not subs:
            name = f"{prefix}{rng.randint(0, 4)}"
            filt = subs[name][1] if name in subs else rng.choice(subjects)
            policy = rng.choice(["all", "new", "last"])
            subs[name] = (await c.subscribe(filt, name, deliver_policy=policy, max_ack_pending=rng.randint(3, 50)),
                          filt)
            held.setdefault(name, [])
            out.append(("sub", name, filt))
        elif op < 0.65:
            name = rng.choice(sorted(subs))
            got = await subs[name][0].fetch(rng.randint(1, 8), 0)
            held[name] += got
            out.append(("fetch", name, [(m.subject, m.data, m.seq, m.metadata.num_delivered) for m in got]))
        elif op < 0.85:
            name = rng.choice(sorted(subs))
            if held[name]:
                m = held[name].pop(rng.randrange(len(held[name])))
                how = rng.choice(["ack", "ack", "nak", "term"])
                await getattr(m, how)()
                out.append((how, name, m.seq))
        else:
            name = rng.choice(sorted(subs))
            i = await c.consumer_info("SMS", name)
            s = await c.stream_info("SMS")
            out.append(("info", i.num_pending, i.num_ack_pending, i.num_redelivered, i.delivered_seq, i.ack_floor,
                        s.messages, s.bytes, s.first_seq, s.last_seq, s.consumers))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_differential_against_python_broker(tmp_path, arun, seed):
    async def run_on(native_):
        sock = f"unix://{tmp_path}/{'n' if native_ else 'p'}{seed}.sock"
        srv = await serve(sock, None, native=native_)
        c = await connect(sock, shared=False)
        try:
            return await _workload(c, seed)
        finally:
            await c.close()
            await srv.close()

    py = arun(run_on(False))
    nat = arun(run_on(True))
    assert len(py) == len(nat)
    for i, (a, b) in enumerate(zip(py, nat)):
        assert a == b, f"op {i}: python={a} native={b}"


def test_native_recovers_python_journal_and_back(tmp_path, arun):
    d = str(tmp_path / "bus")

    async def py_phase():
        bus = await open_file_bus(d)
        for i in range(10):
            await bus.publish(SUBJECT_RAW, f"m{i}".encode())
        sub = await bus.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(6, 0.1)
        for m in got[:4]:
            await m.ack()
        await bus.close()

    async def native_phase():
        sock = f"unix://{tmp_path}/busd.sock"
        srv = await serve(sock, d, native=True)
        c = await connect(sock, shared=False)
        sub = await c.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(100, 0.3)
        info = await c.consumer_info("SMS", "w")
        for m in got[:3]:
            await m.ack()
        await c.publish(SUBJECT_PARSED, b"from-native")
        await asyncio.sleep(0.05)
        await c.close()
        await srv.close()
        return sorted(m.data for m in got), info

    arun(py_phase())
    data, info = arun(native_phase())
    assert data == sorted(f"m{i}".encode() for i in range(4, 10))  # 2 unacked redelivered + 4 new
    assert info.num_ack_pending == 6 and info.num_pending == 0
    # ... and the Python FileLog recovers what the native broker appended
    log = FileLog(d)
    eng = log.open()
    si = eng.stream_info("SMS")
    assert si.messages == 11 and si.last_seq == 11
    assert eng.consumer_info("SMS", "w").num_ack_pending == 3
    log.close()


def test_crash_recovery_torn_tail_and_compaction(tmp_path, arun):
    d = tmp_path / "bus"
    sock = f"unix://{tmp_path}/busd.sock"

    async def phase1():
        b = native.spawn_busd(sock, str(d), compact_bytes=4096)
        c = await connect(sock, shared=False)
        await c.publish_many([(SUBJECT_RAW, b"x" * 100) for _ in range(60)])  # > compact_bytes: compacts
        sub = await c.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(5, 0.2)
        for m in got[:2]:
            await m.ack()
        await c.ping()  # acks are fire-and-forget: a round trip orders them before the crash
        await c.close()
        b.kill()  # SIGKILL: no shutdown flush beyond the per-batch group commit

    arun(phase1())
    segs = sorted(d.glob("journal-*.log"))
    assert len(segs) == 1, segs  # compaction dropped the older segments
    with open(segs[-1], "ab") as f:
        f.write(b"\x50\x00\x00\x00garbage")  # torn frame from a crash mid-write

    async def phase2():
        srv = await serve(sock, str(d), native=True)
        c = await connect(sock, shared=False)
        si = await c.stream_info("SMS")
        sub = await c.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(100, 0.3)
        await c.close()
        await srv.close()
        return si, got

    si, got = arun(phase2())
    assert si.messages == 60
    assert len(got) == 58  # 3 delivered-unacked (redelivered) + 55 never delivered
    assert sorted({m.seq for m in got}) == list(range(3, 61))


def test_sanitizer_build_clean(tmp_path, arun):
    """The broker built with ASan+UBSan runs the differential workload, a journal
    recovery and a graceful shutdown with no sanitizer report (host-side memory /
    UB check; the event loop is single-threaded, so there is no data race to find)."""
    from smsgate_amd.native import build

    san = build.build(sanitize=True)
    sock = f"unix://{tmp_path}/san.sock"
    log = tmp_path / "san.log"

    async def go(seed):
        with open(log, "ab") as f:
            b = native.spawn_busd(sock, str(tmp_path / "data"), binary=san, stderr=f, compact_bytes=16384)
            c = await connect(sock, shared=False)
            out = await _workload(c, seed, n_ops=250, prefix=f"s{seed}-")
            await c.close()
            rc = b.stop()
        return out, rc

    _, rc1 = arun(go(11))
    _, rc2 = arun(go(12))  # second run recovers (and compacts) the first run's journal
    report = log.read_text(errors="replace")
    assert rc1 == 0 and rc2 == 0, report[-2000:]
    assert "ERROR: AddressSanitizer" not in report and "runtime error" not in report, report[-2000:]
