"""Durable bus: journal recovery, broker server/client, multi-process consumers with a crash."""
import asyncio
import multiprocessing as mp
import os
import time

import pytest

from smsgate_amd.bus import SUBJECT_PARSED, SUBJECT_RAW, connect
from smsgate_amd.bus.filelog import FileLog, open_file_bus
from smsgate_amd.bus.server import serve


def test_journal_recovery_redelivers_unacked(tmp_path, arun):
    d = str(tmp_path / "bus")

    async def phase1():
        bus = await open_file_bus(d)
        for i in range(10):
            await bus.publish(SUBJECT_RAW, f"m{i}".encode())
        sub = await bus.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(6, 0.1)
        for m in got[:4]:
            await m.ack()  # 4 acked, 2 delivered-but-unacked, 4 never delivered
        await bus.close()

    async def phase2():
        bus = await open_file_bus(d)
        sub = await bus.subscribe(SUBJECT_RAW, "w")
        got = await sub.fetch(100, 0.2)
        info = await bus.consumer_info("SMS", "w")
        await bus.close()
        return [m.data for m in got], info

    arun(phase1())
    data, info = arun(phase2())
    assert sorted(data) == sorted(f"m{i}".encode() for i in range(4, 10))
    assert info.num_ack_pending == 6 and info.num_pending == 0


def test_journal_torn_tail_and_compaction(tmp_path, arun):
    d = tmp_path / "bus"

    async def go():
        bus = await open_file_bus(str(d))
        for i in range(20):
            await bus.publish(SUBJECT_RAW, b"x" * 100)
        bus._filelog.compact()
        await bus.publish(SUBJECT_RAW, b"after-compact")
        await bus.close()

    arun(go())
    segs = sorted(d.glob("journal-*.log"))
    assert len(segs) == 1
    with open(segs[-1], "ab") as f:  # simulate a crash in the middle of a frame
        f.write(b"\x50\x00\x00\x00garbage")
    log = FileLog(d)
    eng = log.open()
    assert eng.stream_info("SMS").messages == 21
    log.close()


def test_server_client_roundtrip(tmp_path, arun):
    sock = f"unix://{tmp_path}/bus.sock"

    async def go():
        stop = asyncio.Event()
        srv = await serve(sock, str(tmp_path / "data"))
        c1 = await connect(sock, shared=False)
        c2 = await connect(sock, shared=False)
        assert await c1.ping()
        await c1.ensure_stream()
        acks = await c1.publish_many([(SUBJECT_RAW, b"a"), (SUBJECT_RAW, b"b"), (SUBJECT_PARSED, b"p")])
        assert [a.seq for a in acks] == [1, 2, 3]
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
        assert si.messages == 3
        # long-poll wakes up on a publish from another connection
        waiter = asyncio.create_task(s1.fetch(1, 5.0))
        await asyncio.sleep(0.05)
        await c2.publish(SUBJECT_RAW, b"late")
        assert [m.data for m in await waiter] == [b"late"]
        await c1.close()
        await c2.close()
        await srv.close()
        stop.set()

    arun(go())


def _consumer_proc(sock, out_path, crash_after):
    async def go():
        bus = await connect(sock, shared=False)
        sub = await bus.subscribe(SUBJECT_RAW, "workers", ack_wait=0.5)
        n = 0
        idle = 0
        while idle < 10:
            msgs = await sub.fetch(1, 0.2)
            if not msgs:
                idle += 1
                continue
            idle = 0
            m = msgs[0]
            n += 1
            if crash_after and n == crash_after:
                os._exit(3)  # die holding an unacked message
            with open(out_path, "a") as f:
                f.write(m.data.decode() + "\n")
            await m.ack()
        await bus.close()

    asyncio.run(go())


@pytest.mark.slow
@pytest.mark.parametrize("native", [False, True], ids=["python-broker", "native-broker"])
def test_multiprocess_competing_consumers_with_crash(tmp_path, arun, native):
    """N processes share one durable group; one dies mid-message; nothing is lost."""
    if native:
        from smsgate_amd.native import build

        build.build()
    sock = f"unix://{tmp_path}/bus.sock"
    outs = [tmp_path / f"out{i}.txt" for i in range(3)]
    N = 60

    async def go():
        srv = await serve(sock, str(tmp_path / "data"), native=native)
        pub = await connect(sock, shared=False)
        await pub.publish_many([(SUBJECT_RAW, str(i).encode()) for i in range(N)])
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_consumer_proc, args=(sock, str(outs[i]), 5 if i == 0 else 0)) for i in range(3)]
        # the crashing consumer runs alone until it has died holding its 5th message
        # (deterministic: otherwise the others may drain the stream before it gets 5)
        procs[0].start()
        t_end = time.time() + 60
        while procs[0].is_alive() and time.time() < t_end:
            await asyncio.sleep(0.05)
        for p in procs[1:]:
            p.start()
        while any(p.is_alive() for p in procs) and time.time() < t_end:
            await asyncio.sleep(0.1)
        for p in procs:
            p.join(1)
        info = await pub.consumer_info("SMS", "workers")
        await pub.close()
        await srv.close()
        return procs, info

    procs, info = arun(go())
    assert procs[0].exitcode == 3
    seen = []
    for o in outs:
        if o.exists():
            seen += o.read_text().split()
    assert set(seen) == {str(i) for i in range(N)}  # at-least-once: the crashed one's message redelivered
    assert info.num_ack_pending == 0 and info.num_pending == 0
