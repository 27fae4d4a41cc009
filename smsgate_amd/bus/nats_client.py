"""``nats://`` bus: the pipeline's :class:`~smsgate_amd.bus.base.Bus` over the NATS
wire protocol + JetStream API, without nats-py (not on the image).

Lets the services run against an existing NATS JetStream deployment of the
reference (or against our broker's NATS front-end, :mod:`.nats_server`).
Mapping (reference call sites: libs/nats_utils.py:68-129, worker.py:197-224):

* ``publish`` — ``PUB <subject> <inbox>``; the PubAck JSON comes back on the
  inbox (``js.publish``); ``publish_many`` pipelines the publishes;
* ``ensure_stream`` — ``STREAM.INFO`` then ``STREAM.CREATE`` / ``UPDATE``
  (the reference's ensure_stream never created a missing stream — D3);
* ``subscribe`` — a durable **pull** consumer (``CONSUMER.DURABLE.CREATE``,
  explicit acks) instead of the reference's push durable shared by competing
  processes (R3); ``fetch`` = ``CONSUMER.MSG.NEXT`` with ``batch``/``expires``;
* acks — ``+ACK`` / ``-NAK {"delay": ns}`` / ``+TERM`` / ``+WPI`` published to
  the delivery's reply subject;
* ``consumer_info`` / ``stream_info`` — the INFO API responses.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple
from urllib.parse import urlparse

from . import nats_proto as P
from .base import (
    Acker,
    Bus,
    BusError,
    BusUnavailable,
    bus_error,
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

__all__ = ["NatsBus", "connect_nats"]

log = logging.getLogger("nats_bus")


class _ReplyAcker(Acker):
    """Acks a delivery by publishing to its ``$JS.ACK…`` reply subject."""

    __slots__ = ("bus", "reply")

    def __init__(self, bus: "NatsBus", reply: str) -> None:
        self.bus, self.reply = bus, reply

    async def ack(self, stream: str, consumer: str, seq: int) -> None:
        await self.bus._pub(self.reply, b"+ACK")

    async def nak(self, stream: str, consumer: str, seq: int, delay: float) -> None:
        body = b"-NAK" if delay <= 0 else b"-NAK " + P.dumps({"delay": int(delay * P.NS)})
        await self.bus._pub(self.reply, body)

    async def term(self, stream: str, consumer: str, seq: int) -> None:
        await self.bus._pub(self.reply, b"+TERM")

    async def touch(self, stream: str, consumer: str, seq: int) -> None:
        await self.bus._pub(self.reply, b"+WPI")


class _PullSub(Subscription):
    def __init__(self, bus: "NatsBus", stream: str, durable: str) -> None:
        self.bus, self.stream, self.consumer = bus, stream, durable
        self.inbox = P.new_inbox()
        self.queue: "asyncio.Queue[P.Frame]" = asyncio.Queue()
        self.sid = bus._add_sub(self.inbox, self.queue)
        self._closed = False

    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        """>= 1 message as soon as one is available, <= ``batch``.  A NATS pull holds
        until its batch is full or it expires, so: a ``no_wait`` pull for what is
        there, else a long pull for ONE message (in bounded slices so a closed bus
        is noticed), then a ``no_wait`` top-up to ``batch``."""
        got = await self._pull(batch, 0.0)
        if got:
            return got
        slice_s = 5.0
        deadline = None if timeout is None else time.monotonic() + timeout
        while not self._closed:
            left = slice_s if deadline is None else min(slice_s, deadline - time.monotonic())
            if left <= 0.001:
                return []
            got = await self._pull(1, left)
            if got:
                if batch > 1:
                    got += await self._pull(batch - 1, 0.0)
                return got
            if deadline is not None and time.monotonic() >= deadline:
                return []
        return []

    async def _pull(self, batch: int, expires: float) -> List[Msg]:
        while not self.queue.empty():  # drop late status frames of an earlier pull
            self.queue.get_nowait()
        req: Dict[str, Any] = {"batch": batch}
        if expires > 0:
            req["expires"] = int(expires * P.NS)
        else:
            req["no_wait"] = True
        await self.bus._pub(f"{P.API}.CONSUMER.MSG.NEXT.{self.stream}.{self.consumer}", P.dumps(req), self.inbox)
        out: List[Msg] = []
        end = time.monotonic() + expires + 2.0
        while len(out) < batch:
            try:
                f = await asyncio.wait_for(self.queue.get(), max(0.01, end - time.monotonic()))
            except asyncio.TimeoutError:
                break
            if f.op == "HMSG":
                status, text, hdrs = P.decode_headers(f.headers)
                if status is not None:  # 404 no messages / 408 timeout / 409: end of this pull
                    break
            else:
                hdrs = {}
            reply = f.args[2] if len(f.args) > 2 else ""
            meta = P.parse_ack_subject(reply) if reply else None
            if meta is None:
                continue
            out.append(Msg(f.args[0], f.payload,
                           MsgMetadata(meta["stream_seq"], meta["delivered"], meta["timestamp"] / P.NS,
                                       meta["stream"], meta["consumer"]),
                           _ReplyAcker(self.bus, reply), hdrs))
        return out

    async def unsubscribe(self) -> None:
        self._closed = True
        await self.bus._unsub(self.sid)


class NatsBus(Bus):
    def __init__(self, host: str = "127.0.0.1", port: int = 4222, timeout: float = 5.0,
                 stream_config: Optional[StreamConfig] = None) -> None:
        self.host, self.port, self.timeout = host, port, timeout
        self.stream_config = stream_config or default_stream_config()
        self.reader: Optional[asyncio.StreamReader] = None
        self.writer: Optional[asyncio.StreamWriter] = None
        self.server_info: Dict[str, Any] = {}
        self._subs: Dict[str, "asyncio.Queue[P.Frame]"] = {}
        self._next_sid = 1
        self._resp_prefix = P.new_inbox()
        self._resp: Dict[str, asyncio.Future] = {}
        self._wlock = asyncio.Lock()
        self._reader_task: Optional[asyncio.Task] = None
        self._pong: Optional[asyncio.Future] = None
        self._closed = False
        self._stream_cache: Dict[str, str] = {}

    # ------------------------------------------------------------- connection
    async def connect(self) -> "NatsBus":
        self.reader, self.writer = await asyncio.wait_for(asyncio.open_connection(self.host, self.port), self.timeout)
        first = await asyncio.wait_for(P.read_frame(self.reader), self.timeout)
        if first.op != "INFO":
            raise BusError(f"not a NATS server: {first.op}")
        self.server_info = json.loads(first.args[0])
        connect = {"verbose": False, "pedantic": False, "tls_required": False, "name": "smsgate_amd",
                   "lang": "python", "version": "smsgate", "protocol": 1, "headers": True, "no_responders": True}
        self.writer.write(b"CONNECT " + P.dumps(connect) + P.CRLF)
        self._reader_task = asyncio.create_task(self._read_loop())
        self._resp_sid = self._add_sub(self._resp_prefix + ".*", None)
        await self.ping()
        return self

    def _add_sub(self, subject: str, queue: Optional["asyncio.Queue[P.Frame]"]) -> str:
        sid = str(self._next_sid)
        self._next_sid += 1
        self._subs[sid] = queue  # type: ignore[assignment]
        assert self.writer is not None
        self.writer.write(f"SUB {subject} {sid}\r\n".encode())
        return sid

    async def _unsub(self, sid: str) -> None:
        self._subs.pop(sid, None)
        async with self._wlock:
            if self.writer is not None and not self.writer.is_closing():
                self.writer.write(f"UNSUB {sid}\r\n".encode())
                await self.writer.drain()

    async def _pub(self, subject: str, payload: bytes, reply: Optional[str] = None,
                   headers: Optional[bytes] = None) -> None:
        if self.writer is None or self._closed:
            raise BusUnavailable("NATS connection closed")
        async with self._wlock:
            self.writer.write(P.pub_bytes(subject, payload, reply, headers))
            await self.writer.drain()

    async def _read_loop(self) -> None:
        assert self.reader is not None and self.writer is not None
        try:
            while True:
                f = await P.read_frame(self.reader)
                if f.op in ("MSG", "HMSG"):
                    sid = f.args[1]
                    if sid == self._resp_sid:
                        fut = self._resp.pop(f.args[0], None)
                        if fut is not None and not fut.done():
                            fut.set_result(f)
                    else:
                        q = self._subs.get(sid)
                        if q is not None:
                            q.put_nowait(f)
                elif f.op == "PING":
                    self.writer.write(b"PONG\r\n")
                elif f.op == "PONG":
                    if self._pong is not None and not self._pong.done():
                        self._pong.set_result(True)
                elif f.op == "-ERR":
                    log.error("NATS server error: %s", f.args[0] if f.args else "")
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass
        finally:
            self._closed = True
            for fut in self._resp.values():
                if not fut.done():
                    fut.set_exception(BusUnavailable("NATS connection closed"))

    async def request(self, subject: str, payload: bytes, timeout: Optional[float] = None) -> P.Frame:
        token = P.nuid(12)
        inbox = f"{self._resp_prefix}.{token}"
        fut = asyncio.get_running_loop().create_future()
        self._resp[inbox] = fut
        try:
            await self._pub(subject, payload, inbox)
            return await asyncio.wait_for(fut, timeout or self.timeout)
        except asyncio.TimeoutError:
            raise BusUnavailable(f"NATS request on {subject!r} timed out") from None
        finally:
            self._resp.pop(inbox, None)

    async def api(self, what: str, body: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        f = await self.request(f"{P.API}.{what}", P.dumps(body) if body is not None else b"")
        if f.op == "HMSG":
            status, text, _ = P.decode_headers(f.headers)
            if status == 503:
                raise BusUnavailable("JetStream not enabled / no responders")
        return json.loads(f.payload or b"{}")

    # -------------------------------------------------------------------- Bus
    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        cfg = config or self.stream_config
        d = await self.api(f"STREAM.INFO.{cfg.name}")
        if "error" in d:
            d = await self.api(f"STREAM.CREATE.{cfg.name}", P.stream_config_json(cfg))
        elif sorted(d["config"].get("subjects", [])) != sorted(cfg.subjects):
            d = await self.api(f"STREAM.UPDATE.{cfg.name}", P.stream_config_json(cfg))
        if "error" in d:
            raise BusError(d["error"].get("description", "stream error"))
        return self._stream_info(d)

    @staticmethod
    def _stream_info(d: Dict[str, Any]) -> StreamInfo:
        st = d.get("state", {})
        return StreamInfo(config=P.stream_config_from_json(d["config"]), messages=st.get("messages", 0),
                          bytes=st.get("bytes", 0), first_seq=st.get("first_seq", 0),
                          last_seq=st.get("last_seq", 0), consumers=st.get("consumer_count", 0))

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        f = await self.request(subject, data) if not headers else await self._request_h(subject, data, headers)
        if f.op == "HMSG":
            status, text, _ = P.decode_headers(f.headers)
            if status == 503:  # no stream captures it: every publish to it fails alike
                raise BusUnavailable(f"no stream captures subject {subject!r}")
        d = json.loads(f.payload or b"{}")
        if "error" in d:
            raise bus_error(d["error"].get("description", "publish failed"))
        return PubAck(stream=d.get("stream", ""), seq=int(d.get("seq", 0)), duplicate=bool(d.get("duplicate")))

    async def _request_h(self, subject: str, data: bytes, headers: Dict[str, str]) -> P.Frame:
        token = P.nuid(12)
        inbox = f"{self._resp_prefix}.{token}"
        fut = asyncio.get_running_loop().create_future()
        self._resp[inbox] = fut
        try:
            await self._pub(subject, data, inbox, P.encode_headers(headers))
            return await asyncio.wait_for(fut, self.timeout)
        except asyncio.TimeoutError:
            raise BusUnavailable(f"NATS publish on {subject!r} timed out") from None
        finally:
            self._resp.pop(inbox, None)

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        return list(await asyncio.gather(*(self.publish(s, d) for s, d in items)))

    async def _stream_for(self, subject: str) -> str:
        if subject in self._stream_cache:
            return self._stream_cache[subject]
        d = await self.api("STREAM.NAMES", {"subject": subject})
        names = d.get("streams") or []
        if not names:
            raise BusUnavailable(f"no stream for subject {subject!r}")
        self._stream_cache[subject] = names[0]
        return names[0]

    async def subscribe(self, subject: str, durable: str, **opts) -> Subscription:
        stream = await self._stream_for(subject)
        cc = ConsumerConfig(durable=durable, filter_subject=subject, **opts)
        body = {"stream_name": stream, "config": {
            "durable_name": durable, "name": durable, "ack_policy": "explicit",
            "deliver_policy": cc.deliver_policy.value, "filter_subject": subject,
            "ack_wait": int(cc.ack_wait * P.NS), "max_deliver": cc.max_deliver,
            "max_ack_pending": cc.max_ack_pending, "replay_policy": "instant"}}
        d = await self.api(f"CONSUMER.DURABLE.CREATE.{stream}.{durable}", body)
        if "error" in d:
            raise BusError(d["error"].get("description", "consumer create failed"))
        return _PullSub(self, stream, durable)

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        d = await self.api(f"CONSUMER.INFO.{stream}.{durable}")
        if "error" in d:
            raise BusError(d["error"].get("description", "consumer not found"))
        return ConsumerInfo(stream=stream, name=durable, num_pending=d.get("num_pending", 0),
                            num_ack_pending=d.get("num_ack_pending", 0),
                            num_redelivered=d.get("num_redelivered", 0),
                            delivered_seq=d.get("delivered", {}).get("stream_seq", 0),
                            ack_floor=d.get("ack_floor", {}).get("stream_seq", 0),
                            num_waiting=d.get("num_waiting", 0))

    async def stream_info(self, stream: str) -> StreamInfo:
        d = await self.api(f"STREAM.INFO.{stream}")
        if "error" in d:
            raise BusError(d["error"].get("description", "stream not found"))
        return self._stream_info(d)

    async def ping(self) -> bool:
        if self.writer is None or self._closed:
            return False
        self._pong = asyncio.get_running_loop().create_future()
        async with self._wlock:
            self.writer.write(b"PING\r\n")
            await self.writer.drain()
        try:
            await asyncio.wait_for(self._pong, self.timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def is_connected(self) -> bool:
        return self.writer is not None and not self._closed

    async def close(self) -> None:
        self._closed = True
        if self.writer is not None:
            self.writer.close()
            try:
                await self.writer.wait_closed()
            except Exception:  # noqa: BLE001
                pass
        if self._reader_task is not None:
            self._reader_task.cancel()


async def connect_nats(dsn: str, **kw: Any) -> NatsBus:
    u = urlparse(dsn)
    return await NatsBus(u.hostname or "127.0.0.1", u.port or 4222, **kw).connect()
