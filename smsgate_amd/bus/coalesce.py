"""Publish coalescing: many concurrent single publishes -> few ``publish_many`` round trips.

The reference's gateway does one broker round trip per request (plus a
``stream_info`` RPC, nats_utils.py:95-129).  :class:`PublishCoalescer` keeps the
per-request contract -- a request is answered 202 only after ITS message is
persisted (the caller awaits its own PubAck) -- but shares round trips: while one
``publish_many`` is in flight, the publishes that arrive queue up and leave
together in the next one.  At low load a publish goes out alone, immediately (no
timer, no added latency); under load the batch grows with the broker round trip.
"""
from __future__ import annotations

import asyncio
from typing import List, Optional, Tuple

from .base import Bus, PubAck

__all__ = ["PublishCoalescer"]


class PublishCoalescer:
    def __init__(self, bus: Bus, max_batch: int = 512) -> None:
        self.bus = bus
        self.max_batch = max(1, max_batch)
        self._q: List[Tuple[str, bytes, asyncio.Future]] = []
        self._task: Optional[asyncio.Task] = None
        self.round_trips = 0
        self.published = 0

    async def publish(self, subject: str, data: bytes) -> PubAck:
        fut = asyncio.get_running_loop().create_future()
        self._q.append((subject, data, fut))
        if self._task is None:
            # started on the next loop iteration: the requests handled in this one join it
            self._task = asyncio.create_task(self._flush())
        return await fut

    async def _flush(self) -> None:
        try:
            while self._q:
                batch, self._q = self._q[: self.max_batch], self._q[self.max_batch:]
                try:
                    acks = await self.bus.publish_many([(s, d) for s, d, _ in batch])
                except Exception as exc:  # noqa: BLE001 — every request of the batch fails (500)
                    for _, _, f in batch:
                        if not f.done():
                            f.set_exception(exc)
                    continue
                self.round_trips += 1
                self.published += len(batch)
                for (_, _, f), a in zip(batch, acks):
                    if not f.done():
                        f.set_result(a)
        finally:
            self._task = None
