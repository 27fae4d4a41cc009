"""Subject-sharded bus: several brokers act as one bus, each owning some subjects.

The reference runs ONE NATS server for everything (docker-compose.yml:15-27).
One ``smsgate-busd`` event loop carries ≈350 k publish→fetch→ack messages/s with
its journal on (profiles/r02_busd_capacity.jsonl), while a node of 8 GPUs needs
about 3 publishes and 2 deliveries per SMS at ~20 k SMS/s per GPU.  Sharding by
subject keeps every subject's semantics intact (one stream per broker, one
competing consumer group per durable, a durable lives where its subject lives)
and splits the broker work: ``sms.raw`` (ingest → parser) on shard 0; with two
shards the parser's outputs (``sms.parsed`` / ``sms.processing`` / ``sms.failed``
/ ``sms.categorized``) on shard 1; with three (the 8-GPU deployment) one message
per SMS lands on each shard: sms.parsed alone on 1, sms.processing (and the
low-rate subjects) on 2.

DSN: ``sharded+unix:///run/raw.sock,unix:///run/out.sock`` (any member DSNs
:func:`smsgate_amd.bus.connect` accepts, comma separated).
"""
from __future__ import annotations

import asyncio
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

from .base import (
    SUBJECT_PARSED,
    SUBJECT_PROCESSING,
    SUBJECT_RAW,
    Bus,
    BusError,
    ConsumerInfo,
    PubAck,
    StreamConfig,
    StreamInfo,
    Subscription,
)

__all__ = ["ShardedBus", "shard_of"]


def shard_of(subject: str, n: int) -> int:
    """Shard owning ``subject``: ingest (sms.raw) on 0; with 3+ shards sms.parsed
    alone on 1, sms.processing on 2 and the rest spread over 2 .. n-1."""
    if n <= 1 or subject == SUBJECT_RAW:
        return 0
    if n == 2 or subject == SUBJECT_PARSED:
        return 1
    if subject == SUBJECT_PROCESSING:
        return 2
    return 2 + zlib.crc32(subject.encode()) % (n - 2)


class ShardedBus(Bus):
    def __init__(self, members: Sequence[Bus]) -> None:
        if not members:
            raise BusError("sharded bus needs at least one member")
        self.members = list(members)
        self._durables: Dict[Tuple[str, str], int] = {}  # (stream, durable) -> shard

    @classmethod
    async def connect(cls, dsns: Sequence[str], max_age: float) -> "ShardedBus":
        from . import _open

        return cls([await _open(d, max_age) for d in dsns])

    def _bus(self, subject: str) -> Bus:
        return self.members[shard_of(subject, len(self.members))]

    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        infos = await asyncio.gather(*(m.ensure_stream(config) for m in self.members))
        return infos[0]

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        return await self._bus(subject).publish(subject, data, headers)

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        n = len(self.members)
        groups: Dict[int, List[int]] = {}
        for i, (s, _) in enumerate(items):
            groups.setdefault(shard_of(s, n), []).append(i)
        if len(groups) == 1:
            (k, _), = groups.items()
            return await self.members[k].publish_many(items)
        res = await asyncio.gather(*(self.members[k].publish_many([items[i] for i in idx])
                                     for k, idx in groups.items()))
        out: List[Optional[PubAck]] = [None] * len(items)
        for (k, idx), acks in zip(groups.items(), res):
            for i, a in zip(idx, acks):
                out[i] = a
        return out  # type: ignore[return-value]

    async def subscribe(self, subject: str, durable: str, **consumer_opts) -> Subscription:
        k = shard_of(subject, len(self.members))
        sub = await self.members[k].subscribe(subject, durable, **consumer_opts)
        self._durables[(getattr(sub, "stream", None) or "SMS", durable)] = k
        return sub

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        k = self._durables.get((stream, durable))
        if k is not None:
            return await self.members[k].consumer_info(stream, durable)
        for m in self.members:  # a durable created by another client: find its shard
            try:
                info = await m.consumer_info(stream, durable)
            except Exception:  # noqa: BLE001 — not on this shard
                continue
            return info
        raise BusError(f"consumer {durable!r} not found on any shard")

    async def stream_info(self, stream: str) -> StreamInfo:
        infos = await asyncio.gather(*(m.stream_info(stream) for m in self.members))
        first = infos[0]
        first.messages = sum(i.messages for i in infos)
        first.bytes = sum(i.bytes for i in infos)
        return first

    async def ping(self) -> bool:
        return all(await asyncio.gather(*(m.ping() for m in self.members)))

    async def drain(self) -> None:
        await asyncio.gather(*(m.drain() for m in self.members))

    async def close(self) -> None:
        await asyncio.gather(*(m.close() for m in self.members))

    @property
    def is_connected(self) -> bool:
        return all(m.is_connected for m in self.members)
