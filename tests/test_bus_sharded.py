"""ShardedBus: several brokers as one bus, split by subject (sms.raw alone on shard 0)."""
from conftest import drain
from smsgate_amd.bus import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_RAW, MemoryBus
from smsgate_amd.bus.sharded import ShardedBus, shard_of


def test_shard_map():
    assert shard_of(SUBJECT_RAW, 2) == 0 and shard_of(SUBJECT_PARSED, 2) == 1 == shard_of(SUBJECT_FAILED, 2)
    assert {shard_of(s, 4) for s in (SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_FAILED)} <= {1, 2, 3}
    assert shard_of(SUBJECT_PARSED, 1) == 0
    # three shards: one per-SMS message on each broker
    assert [shard_of(s, 3) for s in (SUBJECT_RAW, SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_FAILED)] == [0, 1, 2, 2]


def test_publish_subscribe_ack_across_shards(arun):
    a, b = MemoryBus(), MemoryBus()
    bus = ShardedBus([a, b])

    async def go():
        await bus.ensure_stream()
        acks = await bus.publish_many([(SUBJECT_RAW, b'"r1"'), (SUBJECT_PARSED, b'"p1"'), (SUBJECT_RAW, b'"r2"'),
                                       (SUBJECT_PROCESSING, b'"q1"')])
        sub = await bus.subscribe(SUBJECT_RAW, "parser_worker")
        got = await sub.fetch(10, 0.05)
        for m in got:
            await m.ack()
        info = await bus.consumer_info("SMS", "parser_worker")
        on_a = await drain(a, SUBJECT_PARSED)
        on_b = await drain(b, SUBJECT_PARSED)
        raw_b = await drain(b, SUBJECT_RAW)
        st = await bus.stream_info("SMS")
        return acks, [m.data for m in got], info, on_a, on_b, raw_b, st

    acks, got, info, on_a, on_b, raw_b, st = arun(go())
    assert len(acks) == 4 and all(x is not None for x in acks)
    assert got == [b'"r1"', b'"r2"'] and info.num_ack_pending == 0 and info.num_pending == 0
    assert on_a == [] and on_b == ["p1"] and raw_b == []  # each subject lives on exactly one shard
    assert st.messages == 4


def test_pinned_layout_and_partitioned_subject(arun):
    """``sms.raw`` partitioned over two brokers: publishes are dealt over both, one
    durable name on each, a subscription drains both, consumer_info sums them; the
    other subjects follow their pins / the default member."""
    from smsgate_amd.bus.sharded import Router, parse_members

    dsns, pins, default = parse_members("sms.raw=memory://r0,sms.raw=memory://r1,sms.parsed=memory://p,*=memory://d")
    assert dsns == ["memory://r0", "memory://r1", "memory://p", "memory://d"]
    assert pins == {"sms.raw": [0, 1], "sms.parsed": [2]} and default == [3]
    assert parse_members("memory://a,memory://b")[1] == {}  # positional
    rt = Router(4, pins, default)
    assert rt.members(SUBJECT_PROCESSING) == [3] and rt.members(SUBJECT_RAW) == [0, 1]
    r0, r1, p, d = (MemoryBus() for _ in range(4))
    bus = ShardedBus([r0, r1, p, d], pins, default)

    async def go():
        await bus.ensure_stream()
        await bus.publish_many([(SUBJECT_RAW, f'"r{i}"'.encode()) for i in range(10)])
        await bus.publish(SUBJECT_PARSED, b'"p"')
        await bus.publish(SUBJECT_FAILED, b'"f"')
        sub = await bus.subscribe(SUBJECT_RAW, "parser_worker")
        first = await sub.fetch(4, 0.05)
        info_mid = await bus.consumer_info("SMS", "parser_worker")
        rest = []
        while True:
            got = await sub.fetch(4, 0.05)
            if not got:
                break
            rest += got
        for m in first + rest:
            await m.ack()
        info = await bus.consumer_info("SMS", "parser_worker")
        empty = await sub.fetch(4, 0.05)  # blocking path over both partitions, times out
        per = [(await r.stream_info("SMS")).messages for r in (r0, r1, p, d)]
        return first, rest, info_mid, info, empty, per

    first, rest, info_mid, info, empty, per = arun(go())
    assert sorted(m.data for m in first + rest) == sorted(f'"r{i}"'.encode() for i in range(10))
    assert info_mid.num_ack_pending == 4 and info_mid.num_pending == 6
    assert info.num_ack_pending == 0 and info.num_pending == 0 and empty == []
    assert per == [5, 5, 1, 1]  # raw dealt over both partitions; parsed pinned; failed on the default


def test_partitioned_fetch_survives_a_dead_partition(arun):
    """one failing raw partition must not drop the messages already pulled
    from the healthy ones nor stall them; it is skipped with a backoff, and fetch only
    raises when every partition fails."""
    import pytest

    from smsgate_amd.bus import BusUnavailable

    parts = [MemoryBus() for _ in range(3)]
    pins = {SUBJECT_RAW: [0, 1, 2]}
    bus = ShardedBus(parts + [MemoryBus()], pins, [3])

    async def go():
        await bus.ensure_stream()
        await bus.publish_many([(SUBJECT_RAW, f'"r{i}"'.encode()) for i in range(30)])
        sub = await bus.subscribe(SUBJECT_RAW, "parser_worker")
        async def down(*a, **k):
            raise BusUnavailable("broker down")

        sub.subs[1].fetch = down  # one broker of the partitioned subject goes away
        got = []
        for _ in range(10):
            batch = await sub.fetch(8, 0.05)
            for m in batch:
                await m.ack()
            got += [m.data for m in batch]
        errors = sub.partition_errors
        sub.subs[0].fetch = sub.subs[2].fetch = down
        with pytest.raises(BusUnavailable):
            for _ in range(100):  # outstanding long-polls (<= LONG_POLL s) finish first
                await sub.fetch(8, 0.05)
        return got, errors

    got, errors = arun(go())
    assert len(got) == 20 and len(set(got)) == 20  # the two healthy partitions' 10 + 10 messages
    assert errors >= 1


def test_partitioned_fetch_low_load_latency(arun):
    """A message published to any partition while a consumer long-polls is delivered
    at once (all partitions are polled together), not after (n-1) polling slices."""
    import asyncio
    import time

    parts = [MemoryBus() for _ in range(6)]
    bus = ShardedBus(parts + [MemoryBus()], {SUBJECT_RAW: list(range(6))}, [6])

    async def go():
        await bus.ensure_stream()
        sub = await bus.subscribe(SUBJECT_RAW, "parser_worker")
        lat = []
        for k in range(6):
            async def pub():
                await asyncio.sleep(0.05)
                await parts[k].publish(SUBJECT_RAW, b'"x"')
                return time.monotonic()

            t = asyncio.ensure_future(pub())
            msgs = await sub.fetch(4, 2.0)
            lat.append(time.monotonic() - await t)
            for m in msgs:
                await m.ack()
        await sub.unsubscribe()
        return lat

    lat = arun(go())
    assert max(lat) < 0.03, lat


def test_publishes_are_dealt_per_subject():
    """Interleaved publishes of two partitioned subjects (the parser's sms.parsed /
    sms.processing pairs) reach every partition of each: the dealing turn is per subject."""
    from smsgate_amd.bus.sharded import Router

    rt = Router(5, {"a": [0, 1], "b": [2, 3]}, [4])
    got = [rt.publish_target(s) for _ in range(8) for s in ("a", "b")]
    assert sorted(set(got[0::2])) == [0, 1] and sorted(set(got[1::2])) == [2, 3]
    assert got[0::2].count(0) == 4 and got[1::2].count(2) == 4


def test_bulk_deal_equals_the_per_message_deal():
    """publish_many deals a batch over a subject's partitions in one step per subject
    (Router.deal) -- the same member for every message as one publish_target call per
    message would pick, batch after batch."""
    from smsgate_amd.bus.sharded import Router

    pins = {SUBJECT_RAW: [0, 1, 2], SUBJECT_PARSED: [3, 4]}
    a, b = Router(6, pins, [5]), Router(6, pins, [5])
    for n in (1, 2, 7, 3, 12, 5):
        for subj in (SUBJECT_RAW, SUBJECT_PARSED, SUBJECT_PROCESSING):
            one = [a.publish_target(subj) for _ in range(n)]
            bulk = [None] * n
            for k, sl in b.deal(subj, n):
                for i in range(n)[sl]:
                    bulk[i] = k
            assert bulk == one, (subj, n)
