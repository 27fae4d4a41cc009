"""Bus semantics: durable competing consumers, ack/nak/term, redelivery, retention, stats."""
import asyncio

import pytest
from hypothesis import given, settings, strategies as st

from smsgate_amd.bus import MemoryBus, StreamConfig, connect, subject_matches
from smsgate_amd.bus.base import BusError
from smsgate_amd.bus.engine import Engine


def test_subject_matching():
    assert subject_matches("sms.raw", "sms.raw")
    assert subject_matches("sms.*", "sms.raw")
    assert not subject_matches("sms.*", "sms.raw.x")
    assert subject_matches("sms.>", "sms.raw.x")
    assert not subject_matches("sms.>", "sms")
    assert subject_matches(">", "anything.here")


def test_publish_fetch_ack(arun):
    async def go():
        bus = MemoryBus()
        for i in range(5):
            ack = await bus.publish("sms.raw", f"m{i}".encode())
            assert ack.stream == "SMS" and ack.seq == i + 1
        sub = await bus.subscribe("sms.raw", "w")
        msgs = await sub.fetch(10, timeout=0.1)
        assert [m.data for m in msgs] == [f"m{i}".encode() for i in range(5)]
        info = await bus.consumer_info("SMS", "w")
        assert info.num_ack_pending == 5 and info.num_pending == 0
        for m in msgs:
            await m.ack()
        info = await bus.consumer_info("SMS", "w")
        assert info.num_ack_pending == 0
        assert await sub.fetch(1, timeout=0.05) == []

    arun(go())


def test_filter_and_independent_consumers(arun):
    async def go():
        bus = MemoryBus()
        await bus.publish("sms.raw", b"r")
        await bus.publish("sms.parsed", b"p")
        a = await bus.subscribe("sms.raw", "a")
        b = await bus.subscribe("sms.parsed", "b")
        assert [m.data for m in await a.fetch(5, 0.05)] == [b"r"]
        assert [m.data for m in await b.fetch(5, 0.05)] == [b"p"]
        with pytest.raises(BusError):
            await bus.publish("other.subject", b"x")

    arun(go())


def test_competing_consumers_share_work(arun):
    async def go():
        bus = MemoryBus()
        s1 = await bus.subscribe("sms.raw", "grp")
        s2 = await bus.subscribe("sms.raw", "grp")
        for i in range(10):
            await bus.publish("sms.raw", str(i).encode())
        got1 = await s1.fetch(5, 0.05)
        got2 = await s2.fetch(5, 0.05)
        seqs = sorted(m.seq for m in got1 + got2)
        assert seqs == list(range(1, 11))  # each message to exactly one member
        assert not set(m.seq for m in got1) & set(m.seq for m in got2)

    arun(go())


def test_redelivery_after_ack_wait_and_nak(arun):
    async def go():
        bus = MemoryBus()
        sub = await bus.subscribe("sms.raw", "w", ack_wait=0.05)
        await bus.publish("sms.raw", b"x")
        m1 = (await sub.fetch(1, 0.1))[0]
        assert m1.metadata.num_delivered == 1
        m2 = (await sub.fetch(1, 1.0))[0]  # not acked -> redelivered after ack_wait
        assert m2.seq == m1.seq and m2.metadata.num_delivered == 2
        await m2.nak()
        m3 = (await sub.fetch(1, 0.5))[0]
        assert m3.metadata.num_delivered == 3
        await m3.term()
        assert await sub.fetch(1, 0.15) == []

    arun(go())


def test_max_deliver_drops(arun):
    async def go():
        bus = MemoryBus()
        sub = await bus.subscribe("sms.raw", "w", ack_wait=0.02, max_deliver=2)
        await bus.publish("sms.raw", b"x")
        assert len(await sub.fetch(1, 0.1)) == 1
        assert len(await sub.fetch(1, 0.5)) == 1
        assert await sub.fetch(1, 0.1) == []

    arun(go())


def test_durable_position_survives_rebind(arun):
    async def go():
        bus = MemoryBus()
        s = await bus.subscribe("sms.raw", "w")
        await bus.publish("sms.raw", b"1")
        await bus.publish("sms.raw", b"2")
        m = (await s.fetch(1, 0.05))[0]
        await m.ack()
        await s.unsubscribe()
        s2 = await bus.subscribe("sms.raw", "w")
        assert [x.data for x in await s2.fetch(5, 0.05)] == [b"2"]

    arun(go())


def test_deliver_policy_new(arun):
    async def go():
        bus = MemoryBus()
        await bus.publish("sms.raw", b"old")
        s = await bus.subscribe("sms.raw", "late", deliver_policy="new")
        await bus.publish("sms.raw", b"new")
        assert [x.data for x in await s.fetch(5, 0.05)] == [b"new"]

    arun(go())


def test_retention_max_age_and_max_msgs():
    t = [1000.0]
    eng = Engine(clock=lambda: t[0])
    eng.add_or_update_stream(StreamConfig("S", ["a.*"], max_age=10.0, max_msgs=3))
    from smsgate_amd.bus.base import ConsumerConfig

    eng.add_consumer("S", ConsumerConfig("c", "a.*"))
    for i in range(5):
        eng.store("a.x", str(i).encode())
    info = eng.stream_info("S")
    assert info.messages == 3 and info.first_seq == 3
    assert eng.consumer_info("S", "c").num_pending == 3
    t[0] += 11
    eng.store("a.x", b"fresh")
    assert eng.expire() == 2  # the third old one was evicted by max_msgs on store
    assert eng.stream_info("S").messages == 1
    got = eng.next_batch("S", "c", 10)
    assert [d.msg.data for d in got] == [b"fresh"]


def test_blocking_fetch_wakes_on_publish(arun):
    async def go():
        bus = MemoryBus()
        sub = await bus.subscribe("sms.raw", "w")

        async def later():
            await asyncio.sleep(0.05)
            await bus.publish("sms.raw", b"hi")

        asyncio.create_task(later())
        got = await sub.fetch(1, timeout=2.0)
        assert got and got[0].data == b"hi"

    arun(go())


def test_connect_singleton(arun):
    async def go():
        a = await connect("memory://")
        b = await connect("memory://")
        assert a is b
        assert await a.ping()

    arun(go())


@settings(max_examples=30, deadline=None)
@given(ops=st.lists(st.sampled_from(["pub", "fetch", "ack", "nak", "expire_wait"]), min_size=1, max_size=60))
def test_at_least_once_no_loss(ops):
    """Whatever the interleaving, every published message is eventually acked once."""
    t = [0.0]
    eng = Engine(clock=lambda: t[0])
    eng.add_or_update_stream(StreamConfig("S", ["x"]))
    from smsgate_amd.bus.base import ConsumerConfig

    eng.add_consumer("S", ConsumerConfig("c", "x", ack_wait=1.0))
    published, acked, inflight = set(), set(), []
    for op in ops:
        if op == "pub":
            _, seq = eng.store("x", b"d")
            published.add(seq)
        elif op == "fetch":
            inflight.extend(d.msg.seq for d in eng.next_batch("S", "c", 3))
        elif op == "ack" and inflight:
            s = inflight.pop(0)
            if eng.ack("S", "c", s):
                acked.add(s)
        elif op == "nak" and inflight:
            eng.nak("S", "c", inflight.pop(0))
        elif op == "expire_wait":
            t[0] += 1.5
    # drain: keep fetching and acking (advance time for redeliveries)
    for _ in range(200):
        t[0] += 1.5
        got = eng.next_batch("S", "c", 100)
        for d in got:
            if eng.ack("S", "c", d.msg.seq):
                acked.add(d.msg.seq)
        if not got and eng.consumer_info("S", "c").num_ack_pending == 0:
            break
    assert acked == published
    info = eng.consumer_info("S", "c")
    assert info.num_pending == 0 and info.num_ack_pending == 0
