"""Bus broker process: the NATS-server role for multi-process deployments.

``python -m smsgate_amd bus-server --listen tcp://0.0.0.0:4222 --data ./.bus-data``
serves one journaled engine (:mod:`.filelog`) to any number of service
processes (:class:`~smsgate_amd.bus.client.RemoteBus`) over TCP or a Unix
socket.  Wire format: ``[u32 length][msgpack frame]`` both ways; requests are
``[op, req_id, *args]``, replies ``[req_id, ok, result]``; ``req_id == 0``
means fire-and-forget (acks).  Long-poll ``fetch`` requests run as their own
tasks, so one connection multiplexes many waiting consumers.
"""
from __future__ import annotations

import asyncio
import logging
import struct
from typing import Any, Optional
from urllib.parse import urlparse

import msgpack

from .base import BusError, StreamConfig, default_stream_config
from .memory import MemoryBus

__all__ = ["BusServer", "serve"]

log = logging.getLogger("bus_server")
_LEN = struct.Struct("<I")


def pack(obj: Any) -> bytes:
    body = msgpack.packb(obj, use_bin_type=True)
    return _LEN.pack(len(body)) + body


async def read_frame(reader: asyncio.StreamReader) -> Any:
    hdr = await reader.readexactly(4)
    (n,) = _LEN.unpack(hdr)
    return msgpack.unpackb(await reader.readexactly(n), raw=False, strict_map_key=False)


class BusServer:
    def __init__(self, bus: MemoryBus) -> None:
        self.bus = bus
        self.servers = []
        self.connections = 0

    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.connections += 1
        tasks = set()
        wlock = asyncio.Lock()

        async def reply(rid: int, ok: bool, res: Any) -> None:
            if rid == 0:
                return
            async with wlock:
                writer.write(pack([rid, ok, res]))
                await writer.drain()

        async def run(op: str, rid: int, args: list) -> None:
            try:
                res = await self._dispatch(op, args)
                await reply(rid, True, res)
            except Exception as exc:  # noqa: BLE001 — reported to the caller
                await reply(rid, False, f"{type(exc).__name__}: {exc}")

        try:
            while True:
                frame = await read_frame(reader)
                op, rid, args = frame[0], frame[1], frame[2:]
                if op == "fetch":
                    t = asyncio.create_task(run(op, rid, args))
                    tasks.add(t)
                    t.add_done_callback(tasks.discard)
                else:
                    await run(op, rid, args)
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            for t in tasks:
                t.cancel()
            writer.close()
            self.connections -= 1

    async def _dispatch(self, op: str, a: list) -> Any:
        bus = self.bus
        eng = bus.engine
        if op == "ping":
            return True
        if op == "publish":
            ack = await bus.publish(a[0], a[1], a[2] if len(a) > 2 else None)
            return [ack.stream, ack.seq]
        if op == "publish_many":
            acks = await bus.publish_many([(s, d) for s, d in a[0]])
            return [[x.stream, x.seq] for x in acks]
        if op == "ensure_stream":
            cfg = StreamConfig(**a[0]) if a and a[0] else default_stream_config()
            info = await bus.ensure_stream(cfg)
            return {"name": info.config.name, "messages": info.messages}
        if op == "subscribe":
            subject, durable, opts = a
            sub = await bus.subscribe(subject, durable, **opts)
            return sub.stream  # type: ignore[attr-defined]
        if op == "fetch":
            stream, durable, batch, timeout = a
            from .memory import _MemSub

            sub = _MemSub(bus, stream, durable)
            msgs = await sub.fetch(int(batch), timeout)
            return [[m.subject, m.data, m.seq, m.metadata.num_delivered, m.metadata.timestamp, m.headers or None]
                    for m in msgs]
        if op in ("ack", "term"):
            getattr(eng, op)(a[0], a[1], a[2])
            return None
        if op == "ack_many":
            for s in a[2]:
                eng.ack(a[0], a[1], s)
            return None
        if op == "nak":
            await bus.nak(a[0], a[1], a[2], a[3])
            return None
        if op == "touch":
            eng.touch(a[0], a[1], a[2])
            return None
        if op == "consumer_info":
            i = eng.consumer_info(a[0], a[1])
            return i.__dict__
        if op == "stream_info":
            i = eng.stream_info(a[0])
            d = dict(i.__dict__)
            d["config"] = i.config.__dict__
            return d
        raise BusError(f"unknown op {op!r}")

    async def start(self, listen: str) -> None:
        u = urlparse(listen)
        if u.scheme == "unix":
            srv = await asyncio.start_unix_server(self._handle, path=u.path)
        else:
            srv = await asyncio.start_server(self._handle, host=u.hostname or "127.0.0.1", port=u.port or 4222)
        self.servers.append(srv)
        log.info("bus server listening on %s", listen)

    async def close(self) -> None:
        for s in self.servers:
            s.close()
            await s.wait_closed()
        await self.bus.close()


async def serve(listen: str, data_dir: Optional[str], stop: Optional[asyncio.Event] = None,
                max_age: float = 3 * 24 * 3600.0, nats_listen: Optional[str] = None,
                native: bool = False, http_listen: Optional[str] = None) -> BusServer:
    """One journaled engine behind the msgpack protocol (``listen``) and, optionally,
    the NATS wire protocol (``nats_listen``, :mod:`.nats_server`).

    ``native=True`` runs the C++ broker (:mod:`smsgate_amd.native`, same
    protocol and journal format, its own NATS front-end) as a child process
    instead; the returned object has the same ``close()``.
    """
    if http_listen and not native:
        raise ValueError("--http-listen (native HTTP ingestion) needs --native")
    if native:
        from ..native import spawn_busd

        broker = spawn_busd(listen, data_dir, max_age=max_age, nats_listen=nats_listen or None,
                            http_listen=http_listen or None)
        if stop is not None:
            await stop.wait()
            await broker.close()
        return broker  # type: ignore[return-value]
    if data_dir:
        from .filelog import open_file_bus

        bus = await open_file_bus(data_dir, max_age=max_age)
    else:
        bus = MemoryBus(max_age=max_age)
    server = BusServer(bus)  # type: ignore[arg-type]
    await server.start(listen)
    nats_fe = None
    if nats_listen:
        from .nats_server import NatsFrontend

        u = urlparse(nats_listen)
        nats_fe = NatsFrontend(bus)  # type: ignore[arg-type]
        port = await nats_fe.start(u.hostname or "0.0.0.0", u.port or 4222)
        log.info("NATS protocol front-end on %s:%d", u.hostname, port)
    if stop is not None:
        await stop.wait()
        if nats_fe is not None:
            await nats_fe.close()
        await server.close()
    return server
