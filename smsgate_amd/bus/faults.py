"""Fault injection for any :class:`~smsgate_amd.bus.base.Bus`.

``FaultyBus(inner, ...)`` forwards everything to ``inner`` but can, with seeded
probabilities:

* ``drop_ack`` — swallow a consumer's ``ack`` (the message is redelivered after
  ``ack_wait``: what a crashed worker between "effect done" and "ack" looks like);
* ``nak_ack`` — turn an ``ack`` into an immediate ``nak`` (redelivery at once);
* ``dup_publish`` — publish a message twice (producer retry after a lost PubAck);
* ``delay_publish`` — sleep before each publish (slow broker);
* ``crash_after`` — make a subscription's ``fetch`` raise after N deliveries
  (consumer crash; the Stage loop must survive and unacked work must come back).

Used by the tests to show exactly-once *effects* (idempotent sinks keyed by
``msg_id``) under at-least-once delivery — the property the reference relies on
but never tested (it has no broker tests at all).
"""
from __future__ import annotations

import asyncio
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .base import Acker, Bus, ConsumerInfo, Msg, PubAck, StreamConfig, StreamInfo, Subscription

__all__ = ["FaultyBus", "FaultStats"]


@dataclass
class FaultStats:
    acks_dropped: int = 0
    acks_naked: int = 0
    dup_publishes: int = 0
    crashes: int = 0
    delivered: int = 0
    per_seq: Dict[int, int] = field(default_factory=dict)


class _FaultAcker(Acker):
    def __init__(self, bus: "FaultyBus", inner: Acker) -> None:
        self.bus, self.inner = bus, inner

    async def ack(self, stream: str, consumer: str, seq: int) -> None:
        r = self.bus.rng.random()
        if r < self.bus.drop_ack:
            self.bus.stats.acks_dropped += 1
            return
        if r < self.bus.drop_ack + self.bus.nak_ack:
            self.bus.stats.acks_naked += 1
            await self.inner.nak(stream, consumer, seq, 0.0)
            return
        await self.inner.ack(stream, consumer, seq)

    async def nak(self, stream: str, consumer: str, seq: int, delay: float) -> None:
        await self.inner.nak(stream, consumer, seq, delay)

    async def term(self, stream: str, consumer: str, seq: int) -> None:
        await self.inner.term(stream, consumer, seq)

    async def touch(self, stream: str, consumer: str, seq: int) -> None:
        await self.inner.touch(stream, consumer, seq)


class _FaultSub(Subscription):
    def __init__(self, bus: "FaultyBus", inner: Subscription) -> None:
        self.bus, self.inner = bus, inner
        self.consumer = inner.consumer
        self.delivered = 0

    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        if self.bus.crash_after is not None and self.delivered >= self.bus.crash_after:
            self.bus.crash_after = None  # one crash per bus
            self.bus.stats.crashes += 1
            raise ConnectionError("injected consumer crash")
        got = await self.inner.fetch(batch, timeout)
        out = []
        for m in got:
            self.delivered += 1
            self.bus.stats.delivered += 1
            self.bus.stats.per_seq[m.seq] = self.bus.stats.per_seq.get(m.seq, 0) + 1
            out.append(Msg(m.subject, m.data, m.metadata, _FaultAcker(self.bus, m._acker), m.headers))
        return out

    async def unsubscribe(self) -> None:
        await self.inner.unsubscribe()


class FaultyBus(Bus):
    def __init__(self, inner: Bus, *, drop_ack: float = 0.0, nak_ack: float = 0.0, dup_publish: float = 0.0,
                 delay_publish: float = 0.0, crash_after: Optional[int] = None, seed: int = 0) -> None:
        self.inner = inner
        self.drop_ack, self.nak_ack, self.dup_publish = drop_ack, nak_ack, dup_publish
        self.delay_publish = delay_publish
        self.crash_after = crash_after
        self.rng = random.Random(seed)
        self.stats = FaultStats()

    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        return await self.inner.ensure_stream(config)

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        if self.delay_publish:
            await asyncio.sleep(self.delay_publish)
        ack = await self.inner.publish(subject, data, headers)
        if self.rng.random() < self.dup_publish:
            self.stats.dup_publishes += 1
            await self.inner.publish(subject, data, headers)
        return ack

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        return [await self.publish(s, d) for s, d in items]

    async def subscribe(self, subject: str, durable: str, **consumer_opts) -> Subscription:
        return _FaultSub(self, await self.inner.subscribe(subject, durable, **consumer_opts))

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        return await self.inner.consumer_info(stream, durable)

    async def stream_info(self, stream: str) -> StreamInfo:
        return await self.inner.stream_info(stream)

    async def ping(self) -> bool:
        return await self.inner.ping()

    async def close(self) -> None:
        await self.inner.close()

    def is_connected(self) -> bool:
        return self.inner.is_connected()
