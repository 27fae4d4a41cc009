"""Exactly-once effects under at-least-once delivery, with injected faults
(SURVEY.md §4 items 1 and 6): dropped acks, acks turned into naks, duplicate
publishes and a consumer crash, across the parser and writer stages.  The SQL
sink upserts by msg_id, so every message lands exactly once."""
from __future__ import annotations

import asyncio

from smsgate_amd.bus import SUBJECT_RAW, MemoryBus
from smsgate_amd.bus.faults import FaultyBus
from smsgate_amd.models import RawSMS
from smsgate_amd.parse import ParsePipeline
from smsgate_amd.parse.backends import RegexBackend
from smsgate_amd.services.parser import ParserWorker
from smsgate_amd.services.writer import WriterService
from smsgate_amd.sinks.sql import SqlSink
from smsgate_amd.utils.synth import generate


def test_exactly_once_effects_under_faults(tmp_path, arun):
    items = [s for s in generate(120, seed=77) if s.kind == "purchase"][:40]
    raws = [RawSMS(msg_id=f"m{i}", device_id="d", sender="BANK", date="2025-05-06T00:00:00", body=s.body,
                   source="device") for i, s in enumerate(items)]
    sink = SqlSink(f"sqlite:///{tmp_path}/faults.sqlite")

    async def go():
        bus = FaultyBus(MemoryBus(), drop_ack=0.25, nak_ack=0.1, dup_publish=0.2, crash_after=15, seed=3)
        await bus.ensure_stream()
        for r in raws:
            await bus.publish(SUBJECT_RAW, r.model_dump_json().encode())
        parser = ParserWorker(bus, ParsePipeline(RegexBackend()), batch=8, ack_wait=0.2, stats_interval=0)
        writer = WriterService(bus, [sink], batch=8, ack_wait=0.2, stats_interval=0, retry_min=0.01,
                               retry_max=0.02)
        await parser.start()
        await writer.start()
        for _ in range(300):
            await asyncio.sleep(0.1)
            pi = await bus.consumer_info("SMS", "parser_worker")
            wi = await bus.consumer_info("SMS", "pb_writer")
            if (pi.num_pending == pi.num_ack_pending == 0 and wi.num_pending == wi.num_ack_pending == 0
                    and sink.count() >= len(raws)):
                break
        await parser.stop()
        await writer.stop()
        return bus.stats

    stats = arun(go())
    assert stats.acks_dropped > 0 and stats.acks_naked > 0 and stats.dup_publishes > 0 and stats.crashes == 1
    assert max(stats.per_seq.values()) >= 2  # something really was redelivered
    rows = sink.find([])
    assert sorted(r["msg_id"] for r in rows) == sorted(r.msg_id for r in raws)  # each exactly once
