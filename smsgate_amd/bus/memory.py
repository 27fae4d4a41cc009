"""In-process bus: the :class:`Engine` driven from one asyncio event loop.

Used by tests, by the benchmark and by single-process deployments where all
stages share one loop (``python -m smsgate_amd pipeline``).  Wake-ups are
edge-triggered futures per stream, so an idle consumer costs nothing and a
publish wakes every waiting subscription of the stream once.
"""
from __future__ import annotations

import asyncio
import time
from typing import Dict, List, Optional, Sequence, Tuple

from .base import (
    Acker,
    Bus,
    BusUnavailable,
    ConsumerConfig,
    ConsumerInfo,
    Msg,
    MsgMetadata,
    PubAck,
    StreamConfig,
    StreamInfo,
    Subscription,
    default_stream_config,
)
from .engine import Engine

__all__ = ["MemoryBus"]


class _MemSub(Subscription):
    def __init__(self, bus: "MemoryBus", stream: str, durable: str) -> None:
        self._bus = bus
        self.stream = stream
        self.consumer = durable
        self._closed = False

    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        bus = self._bus
        eng = bus.engine
        deadline = None if timeout is None else time.monotonic() + timeout
        while not self._closed and not bus._closed:
            got = eng.next_batch(self.stream, self.consumer, batch)
            if got:
                return [
                    Msg(
                        d.msg.subject,
                        d.msg.data,
                        MsgMetadata(d.msg.seq, d.num_delivered, d.msg.ts, self.stream, self.consumer),
                        bus,
                        d.msg.headers,
                    )
                    for d in got
                ]
            wait: Optional[float] = None
            if deadline is not None:
                wait = deadline - time.monotonic()
                if wait <= 0:
                    return []
            ready = eng.next_ready_at(self.stream, self.consumer)
            if ready is not None:
                rw = max(0.0, ready - time.time()) + 1e-4
                wait = rw if wait is None else min(wait, rw)
            fut = bus._waiter(self.stream)
            try:
                if wait is None:
                    await asyncio.shield(fut)
                else:
                    await asyncio.wait_for(asyncio.shield(fut), wait)
            except asyncio.TimeoutError:
                pass
        return []

    async def unsubscribe(self) -> None:
        self._closed = True
        self._bus._wake(self.stream)


class MemoryBus(Bus, Acker):
    """A complete :class:`Bus` living inside one process/event loop."""

    def __init__(self, engine: Optional[Engine] = None, *, create_default_stream: bool = True,
                 max_age: float = 3 * 24 * 3600.0) -> None:
        self.engine = engine or Engine()
        self._waiters: Dict[str, asyncio.Future] = {}
        self._closed = False
        self._last_expire = 0.0
        if create_default_stream and not self.engine.streams:
            self.engine.add_or_update_stream(default_stream_config(max_age))

    # -- wake-up plumbing -----------------------------------------------------
    def _waiter(self, stream: str) -> asyncio.Future:
        fut = self._waiters.get(stream)
        if fut is None or fut.done():
            fut = self._waiters[stream] = asyncio.get_running_loop().create_future()
        return fut

    def _wake(self, stream: str) -> None:
        fut = self._waiters.pop(stream, None)
        if fut is not None and not fut.done():
            fut.set_result(None)

    def _maybe_expire(self) -> None:
        now = time.time()
        if now - self._last_expire > 1.0:
            self._last_expire = now
            self.engine.expire(now)

    # -- Bus API ----------------------------------------------------------------
    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        cfg = config or default_stream_config()
        st = self.engine.streams.get(cfg.name)
        if st is not None and sorted(st.cfg.subjects) == sorted(cfg.subjects):
            return self.engine.stream_info(cfg.name)
        return self.engine.add_or_update_stream(cfg)

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        if self._closed:
            raise BusUnavailable("bus closed")
        stream, seq = self.engine.store(subject, bytes(data), headers)
        self._maybe_expire()
        self._wake(stream)
        return PubAck(stream, seq)

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        if self._closed:
            raise BusUnavailable("bus closed")
        stored = self.engine.store_many([(s, bytes(d)) for s, d in items])
        out = [PubAck(stream, seq) for stream, seq in stored]
        touched = {stream for stream, _ in stored}
        self._maybe_expire()
        for s in touched:
            self._wake(s)
        return out

    async def subscribe(self, subject: str, durable: str, **opts) -> Subscription:
        stream = self.engine.stream_for_subject(subject)
        cfg = ConsumerConfig(durable=durable, filter_subject=subject, **opts)
        self.engine.add_consumer(stream, cfg)
        return _MemSub(self, stream, durable)

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        return self.engine.consumer_info(stream, durable)

    async def stream_info(self, stream: str) -> StreamInfo:
        return self.engine.stream_info(stream)

    async def ping(self) -> bool:
        return not self._closed

    async def close(self) -> None:
        self._closed = True
        for s in list(self._waiters):
            self._wake(s)

    @property
    def is_connected(self) -> bool:
        return not self._closed

    # -- Acker --------------------------------------------------------------------
    async def ack(self, stream: str, consumer: str, seq: int) -> None:
        self.engine.ack(stream, consumer, seq)

    async def nak(self, stream: str, consumer: str, seq: int, delay: float) -> None:
        if self.engine.nak(stream, consumer, seq, delay):
            self._wake(stream)

    async def term(self, stream: str, consumer: str, seq: int) -> None:
        self.engine.term(stream, consumer, seq)

    async def touch(self, stream: str, consumer: str, seq: int) -> None:
        self.engine.touch(stream, consumer, seq)
