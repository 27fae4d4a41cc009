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
