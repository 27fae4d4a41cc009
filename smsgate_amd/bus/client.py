"""Client side of the bus broker (:mod:`.server`): ``tcp://`` / ``unix://`` DSNs."""
from __future__ import annotations

import asyncio
import itertools
from collections.abc import Sequence as SequenceABC
from typing import Any, Dict, List, Optional, Sequence, Tuple
from urllib.parse import urlparse

from .base import (
    Acker,
    Bus,
    BusUnavailable,
    bus_error,
    ConsumerInfo,
    Msg,
    PubAck,
    StreamConfig,
    StreamInfo,
    Subscription,
)
from .server import pack, read_frame

__all__ = ["RemoteBus"]


class _RemoteSub(Subscription):
    def __init__(self, bus: "RemoteBus", stream: str, durable: str) -> None:
        self.bus = bus
        self.stream = stream
        self.consumer = durable
        self._closed = False

    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        if self._closed:
            return []
        rows = await self.bus._call("fetch", self.stream, self.consumer, batch, timeout)
        mk, st, co, bus = Msg.delivered, self.stream, self.consumer, self.bus
        return [mk(subj, data, seq, nd, ts, st, co, bus, hdr) for subj, data, seq, nd, ts, hdr in rows]

    async def unsubscribe(self) -> None:
        self._closed = True


class _PubAcks(SequenceABC):
    """The acks of one publish_many, built only when read (the hot publishers -- the
    parser stage, the ingest path -- never read them)."""

    __slots__ = ("_r",)

    def __init__(self, rows) -> None:
        self._r = rows

    def __len__(self) -> int:
        return len(self._r)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [PubAck(s, q) for s, q in self._r[i]]
        s, q = self._r[i]
        return PubAck(s, q)

    def __eq__(self, other) -> bool:
        if not isinstance(other, SequenceABC):
            return NotImplemented
        return list(self) == list(other)


class RemoteBus(Bus, Acker):
    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter, dsn: str) -> None:
        self._r, self._w, self.dsn = reader, writer, dsn
        self._ids = itertools.count(1)
        self._pending: Dict[int, asyncio.Future] = {}
        self._reader_task = asyncio.create_task(self._read_loop())
        self._closed = False
        # acks are coalesced into one ``ack_many`` frame per consumer and loop turn;
        # any other request flushes them first, so ordering is preserved
        self._acks: Dict[Tuple[str, str], List[int]] = {}
        self._ack_flush_scheduled = False

    @classmethod
    async def connect(cls, dsn: str) -> "RemoteBus":
        u = urlparse(dsn)
        if u.scheme == "unix":
            r, w = await asyncio.open_unix_connection(u.path)
        else:
            r, w = await asyncio.open_connection(u.hostname or "127.0.0.1", u.port or 4222)
        return cls(r, w, dsn)

    async def _read_loop(self) -> None:
        try:
            while True:
                rid, ok, res = await read_frame(self._r)
                fut = self._pending.pop(rid, None)
                if fut is not None and not fut.done():
                    if ok:
                        fut.set_result(res)
                    else:
                        fut.set_exception(bus_error(str(res)))
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            self._closed = True
            for fut in self._pending.values():
                if not fut.done():
                    fut.set_exception(BusUnavailable("bus connection closed"))
            self._pending.clear()

    def _flush_acks(self) -> None:
        self._ack_flush_scheduled = False
        if not self._acks or self._closed:
            self._acks.clear()
            return
        for (stream, consumer), seqs in self._acks.items():
            if len(seqs) == 1:
                self._w.write(pack(["ack", 0, stream, consumer, seqs[0]]))
            else:
                self._w.write(pack(["ack_many", 0, stream, consumer, seqs]))
        self._acks.clear()

    async def _call(self, op: str, *args: Any) -> Any:
        if self._closed:
            raise BusUnavailable("bus connection closed")
        self._flush_acks()
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self._pending[rid] = fut
        self._w.write(pack([op, rid, *args]))
        await self._w.drain()
        return await fut

    def _cast(self, op: str, *args: Any) -> None:
        if not self._closed:
            self._flush_acks()
            self._w.write(pack([op, 0, *args]))

    # -- Bus ----------------------------------------------------------------------
    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        await self._call("ensure_stream", config.__dict__ if config else None)
        return await self.stream_info((config.name if config else "SMS"))

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        s, q = await self._call("publish", subject, bytes(data), headers)
        return PubAck(s, q)

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        res = await self._call("publish_many", [[s, d if type(d) is bytes else bytes(d)] for s, d in items])
        return _PubAcks(res)

    async def subscribe(self, subject: str, durable: str, **opts: Any) -> Subscription:
        opts = {k: (v.value if hasattr(v, "value") else v) for k, v in opts.items()}
        stream = await self._call("subscribe", subject, durable, opts)
        return _RemoteSub(self, stream, durable)

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        return ConsumerInfo(**await self._call("consumer_info", stream, durable))

    async def stream_info(self, stream: str) -> StreamInfo:
        d = await self._call("stream_info", stream)
        d["config"] = StreamConfig(**d["config"])
        return StreamInfo(**d)

    async def ping(self) -> bool:
        return bool(await asyncio.wait_for(self._call("ping"), 5.0))

    async def close(self) -> None:
        self._flush_acks()
        self._closed = True
        self._reader_task.cancel()
        self._w.close()

    @property
    def is_connected(self) -> bool:
        return not self._closed

    # -- Acker (fire-and-forget) ---------------------------------------------------
    async def ack(self, stream: str, consumer: str, seq: int) -> None:
        if self._closed:
            return
        self._acks.setdefault((stream, consumer), []).append(seq)
        if not self._ack_flush_scheduled:
            self._ack_flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush_acks)

    async def ack_seqs(self, stream: str, consumer: str, seqs: Sequence[int]) -> None:
        if self._closed:
            return
        self._acks.setdefault((stream, consumer), []).extend(seqs)
        if not self._ack_flush_scheduled:
            self._ack_flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush_acks)

    async def nak(self, stream: str, consumer: str, seq: int, delay: float) -> None:
        self._cast("nak", stream, consumer, seq, delay)

    async def term(self, stream: str, consumer: str, seq: int) -> None:
        self._cast("term", stream, consumer, seq)

    async def touch(self, stream: str, consumer: str, seq: int) -> None:
        self._cast("touch", stream, consumer, seq)
