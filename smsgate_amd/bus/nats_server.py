"""NATS-protocol front-end for the durable broker (the ``nats-server`` role).

``python -m smsgate_amd bus-server --nats-listen tcp://0.0.0.0:4222`` lets NATS
clients — our :class:`~smsgate_amd.bus.nats_client.NatsBus`, or the reference's
nats-py services — talk to the journaled engine (:mod:`.engine`, :mod:`.filelog`)
over the NATS wire protocol.  Supported:

* core: ``INFO``/``CONNECT``/``PING``/``PONG``/``PUB``/``HPUB``/``SUB`` (queue
  groups)/``UNSUB`` and subject routing (``*`` / ``>`` wildcards), so plain
  request/reply between clients works;
* JetStream capture: a publish to a stream subject is stored and, with a reply
  subject, answered with the PubAck JSON ``{"stream", "seq"}``;
* JetStream API: ``STREAM.NAMES/INFO/CREATE/UPDATE/DELETE``, ``CONSUMER.CREATE``
  (+ ``.<filter>`` form) / ``DURABLE.CREATE`` / ``INFO`` / ``DELETE`` /
  ``MSG.NEXT`` (pull: ``batch``, ``expires``, ``no_wait``; 404/408 status
  frames), push consumers (``deliver_subject``: what nats-py's
  ``js.subscribe(subject, durable=...)`` creates, reference worker.py:202);
* acks on ``$JS.ACK.…``: ``+ACK``, ``-NAK`` (optional ``{"delay": ns}``),
  ``+TERM``, ``+WPI``, ``+NXT``; ack-wait redelivery and max_deliver come from the
  engine.

Not implemented (not used by the pipeline): accounts/auth, TLS, clustering,
KV/object stores, flow-control and idle-heartbeat frames, ordered consumers.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Set, Tuple

from . import nats_proto as P
from .base import BusError, ConsumerConfig, DeliverPolicy, subject_matches
from .memory import MemoryBus, _MemSub

__all__ = ["NatsFrontend"]

log = logging.getLogger("nats_frontend")


@dataclass
class _Sub:
    conn: "_Conn"
    sid: str
    subject: str
    queue: Optional[str]


@dataclass(eq=False)  # identity hash: connections live in a set
class _Conn:
    writer: asyncio.StreamWriter
    subs: Dict[str, _Sub] = field(default_factory=dict)
    tasks: Set[asyncio.Task] = field(default_factory=set)
    closed: bool = False

    def send(self, data: bytes) -> None:
        if not self.closed and not self.writer.is_closing():
            self.writer.write(data)


class NatsFrontend:
    def __init__(self, bus: MemoryBus) -> None:
        self.bus = bus
        self.engine = bus.engine
        self.conns: Set[_Conn] = set()
        self.server = None
        self.sid = P.server_id()
        self._cseq: Dict[Tuple[str, str], int] = {}
        self._push: Dict[Tuple[str, str], asyncio.Task] = {}
        self._rr = 0

    # --------------------------------------------------------------- routing
    def _subscribers(self, subject: str) -> List[_Sub]:
        plain: List[_Sub] = []
        groups: Dict[str, List[_Sub]] = {}
        for c in self.conns:
            for s in c.subs.values():
                if subject_matches(s.subject, subject):
                    if s.queue:
                        groups.setdefault(s.queue, []).append(s)
                    else:
                        plain.append(s)
        for members in groups.values():
            self._rr += 1
            plain.append(members[self._rr % len(members)])
        return plain

    def route(self, subject: str, payload: bytes, reply: Optional[str] = None,
              headers: Optional[bytes] = None) -> int:
        subs = self._subscribers(subject)
        for s in subs:
            s.conn.send(P.msg_bytes(subject, s.sid, payload, reply, headers))
        return len(subs)

    def _status(self, reply: str, code: int, text: str) -> None:
        self.route(reply, b"", None, P.encode_headers(None, f"{code} {text}"))

    # ------------------------------------------------------------ connections
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        conn = _Conn(writer)
        self.conns.add(conn)
        host, port = (writer.get_extra_info("sockname") or ("127.0.0.1", 4222))[:2]
        info = {"server_id": self.sid, "server_name": "smsgate_amd", "version": "2.10.0", "proto": 1,
                "go": "n/a", "host": str(host), "port": int(port) if isinstance(port, int) else 4222,
                "headers": True, "max_payload": P.MAX_PAYLOAD, "jetstream": True}
        conn.send(b"INFO " + P.dumps(info) + P.CRLF)
        try:
            while True:
                f = await P.read_frame(reader)
                if f.op in ("PUB", "HPUB"):
                    await self._on_pub(conn, f)
                elif f.op == "SUB":
                    subject, sid = f.args[0], f.args[-1]
                    queue = f.args[1] if len(f.args) == 3 else None
                    conn.subs[sid] = _Sub(conn, sid, subject, queue)
                elif f.op == "UNSUB":
                    conn.subs.pop(f.args[0], None)
                elif f.op == "PING":
                    conn.send(b"PONG\r\n")
                elif f.op in ("CONNECT", "PONG", ""):
                    pass
                else:
                    conn.send(b"-ERR 'Unknown Protocol Operation'\r\n")
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.LimitOverrunError):
            pass
        finally:
            conn.closed = True
            self.conns.discard(conn)
            for t in conn.tasks:
                t.cancel()
            writer.close()

    def _spawn(self, conn: _Conn, coro) -> None:
        t = asyncio.create_task(coro)
        conn.tasks.add(t)
        t.add_done_callback(conn.tasks.discard)

    async def _on_pub(self, conn: _Conn, f: P.Frame) -> None:
        subject = f.args[0]
        reply = f.args[1] if len(f.args) > 1 else None
        if subject.startswith(P.API + "."):
            self._spawn(conn, self._api(subject[len(P.API) + 1:], f.payload, reply))
            return
        if subject.startswith(P.ACK_PREFIX):
            await self._on_ack(subject, f.payload)
            if reply:
                self.route(reply, b"")
            return
        hdrs = P.decode_headers(f.headers)[2] if f.headers else None
        try:
            self.engine.stream_for_subject(subject)
            captured = True
        except BusError:
            captured = False
        if captured:
            ack = await self.bus.publish(subject, f.payload, hdrs)
            if reply:
                self.route(reply, P.dumps({"stream": ack.stream, "seq": ack.seq}))
        n = self.route(subject, f.payload, reply if not captured else None, f.headers or None)
        if not captured and n == 0 and reply:
            self._status(reply, 503, "No Responders")

    async def _on_ack(self, subject: str, body: bytes) -> None:
        meta = P.parse_ack_subject(subject)
        if meta is None:
            return
        s, c, seq = meta["stream"], meta["consumer"], meta["stream_seq"]
        try:
            if body in (b"", b"+ACK", b"+NXT") or body.startswith(b"+NXT"):
                await self.bus.ack(s, c, seq)
            elif body.startswith(b"-NAK"):
                delay = 0.0
                rest = body[4:].strip()
                if rest:
                    try:
                        delay = float(json.loads(rest).get("delay", 0)) / P.NS
                    except ValueError:
                        pass
                await self.bus.nak(s, c, seq, delay)
            elif body.startswith(b"+TERM"):
                await self.bus.term(s, c, seq)
            elif body.startswith(b"+WPI"):
                await self.bus.touch(s, c, seq)
        except BusError as exc:
            log.debug("ack on %s ignored: %s", subject, exc)

    # --------------------------------------------------------------- JetStream
    def _ack_subject(self, stream: str, consumer: str, m) -> str:
        k = (stream, consumer)
        self._cseq[k] = self._cseq.get(k, 0) + 1
        return (f"{P.ACK_PREFIX}{stream}.{consumer}.{m.metadata.num_delivered}.{m.seq}.{self._cseq[k]}."
                f"{int(m.metadata.timestamp * P.NS)}.0")

    def _stream_json(self, name: str) -> Dict[str, Any]:
        si = self.engine.stream_info(name)
        return {"type": "io.nats.jetstream.api.v1.stream_info_response",
                "config": P.stream_config_json(si.config), "created": "1970-01-01T00:00:00Z",
                "state": {"messages": si.messages, "bytes": si.bytes, "first_seq": si.first_seq,
                          "last_seq": si.last_seq, "consumer_count": si.consumers}}

    def _consumer_json(self, stream: str, durable: str) -> Dict[str, Any]:
        ci = self.engine.consumer_info(stream, durable)
        cfg = self.engine.streams[stream].consumers[durable].cfg
        cseq = self._cseq.get((stream, durable), 0)
        return {"type": "io.nats.jetstream.api.v1.consumer_info_response", "stream_name": stream,
                "name": durable, "created": "1970-01-01T00:00:00Z",
                "config": {"durable_name": durable, "name": durable, "ack_policy": "explicit",
                           "deliver_policy": cfg.deliver_policy.value, "filter_subject": cfg.filter_subject,
                           "ack_wait": int(cfg.ack_wait * P.NS), "max_deliver": cfg.max_deliver,
                           "max_ack_pending": cfg.max_ack_pending, "replay_policy": "instant"},
                "delivered": {"consumer_seq": cseq, "stream_seq": ci.delivered_seq},
                "ack_floor": {"consumer_seq": 0, "stream_seq": ci.ack_floor},
                "num_ack_pending": ci.num_ack_pending, "num_redelivered": ci.num_redelivered,
                "num_waiting": ci.num_waiting, "num_pending": ci.num_pending}

    async def _api(self, what: str, body: bytes, reply: Optional[str]) -> None:
        try:
            res = await self._api_call(what, body, reply)
        except BusError as exc:
            msg = str(exc)
            code, err = (404, 10059 if "stream" in msg and "not found" in msg else 10014) if "not found" in msg \
                else (400, 10058)
            res = P.api_error(code, err, msg)
        except (ValueError, KeyError) as exc:
            res = P.api_error(400, 10025, f"bad request: {exc}")
        if res is not None and reply:
            self.route(reply, P.dumps(res))

    async def _api_call(self, what: str, body: bytes, reply: Optional[str]) -> Optional[Dict[str, Any]]:
        t = what.split(".")
        req = json.loads(body) if body.strip().startswith(b"{") else {}
        if t[0] == "INFO":
            return {"type": "io.nats.jetstream.api.v1.account_info_response", "streams": len(self.engine.streams)}
        if t[0] == "STREAM":
            op = t[1]
            if op == "NAMES" or op == "LIST":
                subj = req.get("subject")
                names = [n for n, st in self.engine.streams.items()
                         if not subj or any(subject_matches(p, subj) or subject_matches(subj, p)
                                            for p in st.cfg.subjects)]
                if op == "LIST":
                    return {"total": len(names), "offset": 0, "limit": 1024,
                            "streams": [self._stream_json(n) for n in names]}
                return {"total": len(names), "offset": 0, "limit": 1024, "streams": names}
            name = t[2]
            if op == "INFO":
                return self._stream_json(name)
            if op in ("CREATE", "UPDATE"):
                cfg = P.stream_config_from_json(req or {"name": name})
                if op == "UPDATE" and name not in self.engine.streams:
                    raise BusError(f"stream {name!r} not found")
                await self.bus.ensure_stream(cfg)
                return self._stream_json(name)
            if op == "DELETE":
                self.engine.streams.pop(name, None)
                self.engine._route_cache.clear()
                return {"success": True}
        if t[0] == "CONSUMER":
            op = t[1]
            if op in ("CREATE", "DURABLE"):
                if op == "DURABLE":  # DURABLE.CREATE.<stream>.<durable>
                    stream, name = t[3], t[4]
                else:  # CREATE.<stream>[.<consumer>[.<filter>]]
                    stream = t[2]
                    name = t[3] if len(t) > 3 else None
                c = req.get("config", {})
                durable = c.get("durable_name") or c.get("name") or name
                if not durable:
                    raise ValueError("ephemeral consumers are not supported")
                cc = ConsumerConfig(durable=durable, filter_subject=c.get("filter_subject") or ">",
                                    ack_wait=float(c.get("ack_wait", 30 * P.NS)) / P.NS,
                                    max_deliver=int(c.get("max_deliver", -1)),
                                    deliver_policy=DeliverPolicy(c.get("deliver_policy", "all")
                                                                 if c.get("deliver_policy", "all") in ("all", "new", "last")
                                                                 else "all"),
                                    max_ack_pending=int(c.get("max_ack_pending", 65536) or 65536))
                self.engine.add_consumer(stream, cc)
                if c.get("deliver_subject"):
                    self._start_push(stream, durable, c["deliver_subject"])
                return self._consumer_json(stream, durable)
            if op == "INFO":
                return self._consumer_json(t[2], t[3])
            if op == "DELETE":
                task = self._push.pop((t[2], t[3]), None)
                if task:
                    task.cancel()
                self.engine.delete_consumer(t[2], t[3])
                return {"success": True}
            if op == "MSG" and t[2] == "NEXT":
                await self._pull(t[3], t[4], body, reply)
                return None
        raise ValueError(f"unsupported API {what}")

    async def _pull(self, stream: str, durable: str, body: bytes, reply: Optional[str]) -> None:
        if not reply:
            return
        self.engine.consumer_info(stream, durable)  # raises if missing
        b = body.strip()
        if b.startswith(b"{"):
            req = json.loads(b)
        elif b:
            req = {"batch": int(b)}
        else:
            req = {"batch": 1}
        batch = max(1, int(req.get("batch", 1)))
        expires = float(req.get("expires", 0)) / P.NS
        no_wait = bool(req.get("no_wait")) or expires <= 0
        sub = _MemSub(self.bus, stream, durable)
        sent = 0
        deadline = time.monotonic() + (0.0 if no_wait else expires)
        while sent < batch:
            left = deadline - time.monotonic()
            got = await sub.fetch(batch - sent, 0.0 if (no_wait or left <= 0) else left)
            if not got:
                break
            for m in got:
                self.route(reply, m.data, self._ack_subject(stream, durable, m),
                           P.encode_headers(m.headers) if m.headers else None)
            sent += len(got)
            if no_wait:
                break
        if sent < batch:  # end the request: a client waits for the batch or a status frame
            if no_wait:
                self._status(reply, 404, "No Messages")
            else:
                self._status(reply, 408, "Request Timeout")

    def _start_push(self, stream: str, durable: str, deliver: str) -> None:
        key = (stream, durable)
        if key in self._push and not self._push[key].done():
            return

        async def run() -> None:
            sub = _MemSub(self.bus, stream, durable)
            while True:
                if not self._subscribers(deliver):
                    await asyncio.sleep(0.05)
                    continue
                got = await sub.fetch(256, 1.0)
                for m in got:
                    if self.route(deliver, m.data, self._ack_subject(stream, durable, m),
                                  P.encode_headers(m.headers) if m.headers else None) == 0:
                        await self.bus.nak(stream, durable, m.seq, 0.0)

        self._push[key] = asyncio.create_task(run())

    # ------------------------------------------------------------- lifecycle
    async def start(self, host: str = "127.0.0.1", port: int = 4222) -> int:
        self.server = await asyncio.start_server(self._handle, host, port, limit=P.MAX_PAYLOAD + 1024)
        return self.server.sockets[0].getsockname()[1]

    async def close(self) -> None:
        for t in self._push.values():
            t.cancel()
        if self.server is not None:
            self.server.close()
            await self.server.wait_closed()
        for c in list(self.conns):
            c.closed = True
            c.writer.close()
