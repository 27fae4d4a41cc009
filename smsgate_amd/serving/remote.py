"""Engine server (GPU process) and client (parser processes).

Topology per MI355X (see ``bench.py`` and ``python -m smsgate_amd engine-server``):

    parser worker 1 ─┐                       ┌──────────────────────────────┐
    parser worker 2 ─┼── pipes / unix socket ─► EngineServer (GPU process)  │
    parser worker K ─┘   token ids ⇄ ids     │  continuous batching engine  │
                                             └──────────────────────────────┘

The GPU process does nothing but schedule the engine: its Python work per
message is a few array slices, so the decode graphs are replayed back to back
while the CPU-heavy work — tokenisation, detokenisation, post-processing,
validation, bus I/O — runs in K parser processes with their own interpreters
(no shared GIL). Parser workers must be started before the GPU process
initialises the GPU (no exec after GPU init on this platform).
"""
from __future__ import annotations

import asyncio
import itertools
import queue
import selectors
import threading
import time
import weakref
from dataclasses import dataclass, field
from multiprocessing.connection import Connection
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

from . import protocol as P
from .protocol import PackedAnswer
from .qa import null_rejection

__all__ = ["EngineServer", "RemoteEngineClient"]


@dataclass
class _Req:
    conn_idx: int
    req_id: int
    out: List[Any]
    left: int


class EngineServer:
    def __init__(self, engine, conns: Sequence[Connection] = (),
                 on_control: Optional[Callable[[int, Any], None]] = None) -> None:
        self.engine = engine
        self.conns: List[Optional[Connection]] = list(conns)
        self.on_control = on_control
        self.reqs: Dict[tuple, _Req] = {}
        self.served = 0
        self._packed = callable(getattr(engine, "submit_packed", None))
        # one persistent selector over the live connections (multiprocessing's wait()
        # builds and tears down a selector per call: ~3 us per message of the poll loop)
        self._sel = selectors.DefaultSelector()
        for i, c in enumerate(self.conns):
            self._sel.register(c, selectors.EVENT_READ, i)
        # responses leave through sender threads, one per connection: a parser process
        # that is slow to read (its reader thread waits for the GIL) filled its socket and
        # blocked the engine loop inside send_bytes -- 1.7 s of a 3.2 s phase with the GPU
        # idle behind it -- and with one shared sender it would hold back every other
        # connection's responses the same way
        self._senders: Dict[int, "queue.SimpleQueue"] = {}  # id(connection) -> its FIFO
        self._senders_lock = threading.Lock()
        # connections gone: late frames for them are discarded.  Weak: a dropped connection
        # is closed by its sender thread once its queued frames are out, then collected
        self._dropped: "weakref.WeakSet[Connection]" = weakref.WeakSet()

    def _send(self, c: Connection, frame: bytes) -> None:
        """Queue ``frame`` for ``c`` (its frames leave in order, on its own thread)."""
        q = self._senders.get(id(c))
        if q is None:
            with self._senders_lock:
                if c in self._dropped:  # (no new sender thread for a connection that is gone)
                    return
                q = self._senders.get(id(c))
                if q is None:
                    q = self._senders[id(c)] = queue.SimpleQueue()
                    threading.Thread(target=self._send_loop, args=(c, q), name="engine-send",
                                     daemon=True).start()
        q.put(frame)

    @staticmethod
    def _send_loop(c: Connection, q: "queue.SimpleQueue") -> None:
        dead = False
        while True:
            frame = q.get()
            if frame is None:  # dropped: the frames queued before are out, release the socket
                try:
                    c.close()
                except OSError:
                    pass
                return
            if isinstance(frame, threading.Event):  # a flush marker
                frame.set()
                continue
            if dead:
                continue
            try:
                c.send_bytes(frame)
            except (OSError, EOFError, ValueError):  # the client went away: drop what follows
                dead = True

    def flush(self, timeout: float = 30.0, conns: Optional[Sequence[Connection]] = None) -> bool:
        """Wait until every queued frame (of ``conns``, default all connections) has been
        handed to the sockets.  False (and a log line) when ``timeout`` ran out first: a
        parser that stalls without disconnecting must not hold the caller silently."""
        with self._senders_lock:
            if conns is None:
                queues = list(self._senders.values())
            else:
                queues = [q for q in (self._senders.get(id(c)) for c in conns) if q is not None]
        marks = []
        for q in queues:
            ev = threading.Event()
            q.put(ev)
            marks.append(ev)
        t_end = time.monotonic() + timeout
        ok = all([ev.wait(max(0.0, t_end - time.monotonic())) for ev in marks])
        if not ok:
            import logging

            logging.getLogger(__name__).warning("engine server: %d of %d connection(s) did not drain within %.1f s",
                                                sum(not ev.is_set() for ev in marks), len(marks), timeout)
        return ok

    def add_connection(self, conn: Connection) -> int:
        self.conns.append(conn)
        self._sel.register(conn, selectors.EVENT_READ, len(self.conns) - 1)
        return len(self.conns) - 1

    def _drop(self, idx: int) -> None:
        c = self.conns[idx]
        self.conns[idx] = None
        if c is not None:
            try:
                self._sel.unregister(c)
            except (KeyError, ValueError, OSError):
                pass
            with self._senders_lock:
                q = self._senders.pop(id(c), None)
                self._dropped.add(c)
            if q is not None:  # its sender closes it after the frames already queued
                q.put(None)
            else:  # no sender thread: nothing queued, close it now
                try:
                    c.close()
                except OSError:
                    pass

    def send_control(self, idx: int, obj: Any) -> None:
        c = self.conns[idx]
        if c is not None:
            self._send(c, P.pack_control(obj))
            # control frames (harness commands) leave before the caller goes on; only this
            # connection's queue is waited for (a broadcast over N connections would
            # otherwise wait N times on every stalled parser)
            self.flush(conns=[c])

    def _live(self) -> List[Connection]:
        return [c for c in self.conns if c is not None]

    def poll(self, timeout: Optional[float]) -> None:
        t0 = time.perf_counter()
        try:
            self._poll(timeout)
        finally:
            st = getattr(self.engine, "stats", None)
            if st is not None and hasattr(st, "server_poll_s"):
                st.server_poll_s += time.perf_counter() - t0

    def _poll(self, timeout: Optional[float]) -> None:
        if not self._sel.get_map():
            if timeout:
                time.sleep(min(timeout, 0.01))
            return
        for key, _ in self._sel.select(timeout):
            idx, c = key.data, key.fileobj
            while True:
                try:
                    buf = c.recv_bytes()
                except (EOFError, OSError):
                    self._drop(idx)
                    break
                k = P.kind(buf)
                if k == b"Q":
                    if self._packed:  # the whole request is one engine unit (QAEngine.submit_packed)
                        _, rid, lens, flat = P.unpack_arrays(buf)
                        if not len(lens):
                            self._send(c, P.pack_ids(b"R", rid, []))
                        else:
                            try:
                                self.engine.submit_packed((idx, rid), lens, flat)
                            except ValueError as exc:  # a malformed request fails alone
                                self._send(c, P.pack_error(rid, repr(exc)))
                        if not c.poll():
                            break
                        continue
                    _, rid, seqs = P.unpack_id_arrays(buf)
                    if not seqs:
                        self._send(c, P.pack_ids(b"R", rid, []))
                    else:
                        self.reqs[(idx, rid)] = _Req(idx, rid, [None] * len(seqs), len(seqs))
                        self.engine.submit_ids([((idx, rid, i), s) for i, s in enumerate(seqs)])
                elif k == b"C" and self.on_control is not None:
                    self.on_control(idx, P.unpack_control(buf))
                if not c.poll():
                    break

    def step(self) -> None:
        try:
            finished = self.engine.step(raw=True)
        except Exception as exc:  # fail every waiting request loudly
            keys = list(self.reqs)
            if self._packed:  # whole requests queued / in flight in the engine
                units = list(self.engine.waiting)
                for b in getattr(self.engine, "_inflight", ()):
                    units += list(getattr(b, "units", None) or [])
                keys += [u.key for u in units if getattr(u, "packed", False)]
            for idx, rid in dict.fromkeys(keys):  # (a split request's parts share one key)
                c = self.conns[idx]
                if c is not None:
                    self._send(c, P.pack_error(rid, repr(exc)))
            self.reqs.clear()
            self.engine.waiting.clear()
            self.engine.active.clear()
            self.engine._pending = None
            if hasattr(self.engine, "_inflight"):
                self.engine._inflight.clear()
            raise
        t0 = time.perf_counter()
        for key, toks in finished:
            if isinstance(toks, PackedAnswer):  # a whole request: its response frame as is
                idx, rid = key
                c = self.conns[idx]
                if c is not None:
                    self._send(c, P.pack_arrays(b"R", rid, toks.lens, toks.flat))
                self.served += len(toks.lens)
                continue
            idx, rid, i = key
            r = self.reqs.get((idx, rid))
            if r is None:
                continue
            r.out[i] = toks
            r.left -= 1
            if r.left == 0:
                del self.reqs[(idx, rid)]
                c = self.conns[idx]
                if c is not None:
                    lens = np.fromiter((len(t) for t in r.out), dtype=np.uint16, count=len(r.out))
                    flat = np.concatenate(r.out) if r.out else np.zeros(0, np.int32)
                    self._send(c, P.pack_arrays(b"R", rid, lens, flat))
                self.served += len(r.out)
        st = getattr(self.engine, "stats", None)
        if st is not None and hasattr(st, "server_send_s"):
            st.server_send_s += time.perf_counter() - t0

    def serve_until(self, pred: Callable[[], bool]) -> None:
        while not pred():
            self.poll(0 if self.engine.busy() else 0.002)
            if self.engine.busy():
                self.step()

    def serve_forever(self) -> None:
        self.serve_until(lambda: not self._live() and not self.engine.busy())

    def serve_listener(self, address: str, stop: Optional[threading.Event] = None) -> None:
        """Accept parser processes on ``address`` (a unix socket path) and serve them
        until ``stop`` is set — the standalone ``engine-server`` process."""
        from multiprocessing.connection import Listener

        incoming: "queue.Queue[Connection]" = queue.Queue()
        listener = Listener(address, family="AF_UNIX")

        def accept_loop() -> None:
            while stop is None or not stop.is_set():
                try:
                    incoming.put(listener.accept())
                except OSError:
                    return

        threading.Thread(target=accept_loop, name="engine-accept", daemon=True).start()

        def pred() -> bool:
            while not incoming.empty():
                self.add_connection(incoming.get_nowait())
            return stop is not None and stop.is_set()

        try:
            self.serve_until(pred)
        finally:
            listener.close()
            self.flush(5.0)  # answers already produced reach their clients
            # clients see EOF (and reconnect to the next server): _drop closes each
            # connection, on its sender thread once that thread's frames are out
            for i, c in enumerate(self.conns):
                if c is not None:
                    self._drop(i)


class RemoteEngineClient:
    """Async client: tokenises, ships ids, awaits ids, detokenises into answers.

    ``connector`` (a zero-argument callable returning a fresh
    :class:`~multiprocessing.connection.Connection`) makes the client survive an
    engine-server restart: when the socket closes, every in-flight request fails
    with :class:`~smsgate_amd.parse.backends.base.BackendUnavailable` (a
    transient error: the parser stage naks the batch and retries it later
    instead of dead-lettering its messages), and the next request reconnects.
    """

    def __init__(self, conn: Optional[Connection] = None, tokenizer=None, max_body_tokens: int = 128,
                 connector: Optional[Callable[[], Connection]] = None,
                 request_timeout: Optional[float] = 120.0) -> None:
        from ..models.tokenizer import load_tokenizer
        from .fsm import DEFAULT_FIELDS

        if conn is None and connector is None:
            raise ValueError("RemoteEngineClient needs a connection or a connector")
        self.connector = connector
        self.tok = tokenizer or load_tokenizer()
        # native encoder / decoder (native/csrc/tokfast.cpp, id-for-id the library's);
        # None when the extension is not built -> the library path
        from ..models.fasttok import load_fast_tokenizer

        self.fast = load_fast_tokenizer() if tokenizer is None else None
        self.fields = [f.name for f in DEFAULT_FIELDS]
        self.max_body = max_body_tokens
        self._ids = itertools.count(1)
        # rid -> (future, loop, connection it was sent on): a dying connection's reader
        # fails exactly its own requests (a request already sent on the next connection
        # is never swept by the old reader)
        self._pending: Dict[int, Any] = {}
        self._plock = threading.Lock()
        self.request_timeout = request_timeout
        self._send_lock = threading.Lock()
        self._conn_lock = threading.Lock()
        self.control: "queue.Queue[Any]" = queue.Queue()
        self.conn: Optional[Connection] = None
        self.reconnects = 0
        if conn is None:
            try:
                conn = connector()  # type: ignore[misc]
            except OSError:  # engine not up yet: the first request connects (or naks)
                return
        self._attach(conn)

    def _attach(self, conn: Connection) -> None:
        self.conn = conn
        self._reader = threading.Thread(target=self._read_loop, args=(conn,), name="engine-client", daemon=True)
        self._reader.start()

    def _unavailable(self, why: str):
        from ..parse.backends.base import BackendUnavailable

        return BackendUnavailable(why)

    def _connection(self) -> Connection:
        with self._conn_lock:
            if self.conn is not None:
                return self.conn
            if self.connector is None:
                raise self._unavailable("engine server closed (no connector to reconnect)")
            try:
                conn = self.connector()
            except OSError as exc:
                raise self._unavailable(f"engine server unreachable: {exc}") from exc
            self.reconnects += 1
            self._attach(conn)
            return conn

    def _read_loop(self, conn: Connection) -> None:
        while True:
            try:
                buf = conn.recv_bytes()
            except (EOFError, OSError):
                # detach first, then sweep: a request registered after the sweep sees
                # self.conn is not its connection and fails itself (extract)
                with self._conn_lock:
                    if self.conn is conn:
                        self.conn = None
                with self._plock:
                    mine = [rid for rid, e in self._pending.items() if e[2] is conn]
                    ents = [self._pending.pop(rid) for rid in mine]
                for fut, loop, _ in ents:
                    loop.call_soon_threadsafe(self._set_exc, fut, self._unavailable("engine server closed"))
                self.control.put(None)
                return
            k = P.kind(buf)
            if k == b"R":
                rid = P.req_id(buf)
                with self._plock:
                    ent = self._pending.pop(rid, None)
                if ent is not None:
                    fut, loop, _ = ent
                    # the raw response: decoded on the event loop (natively when built)
                    loop.call_soon_threadsafe(self._set_res, fut, buf)
            elif k == b"E":
                rid, msg = P.unpack_error(buf)
                with self._plock:
                    ent = self._pending.pop(rid, None)
                if ent is not None:
                    fut, loop, _ = ent
                    loop.call_soon_threadsafe(self._set_exc, fut, RuntimeError(msg))
            elif k == b"C":
                self.control.put(P.unpack_control(buf))

    @staticmethod
    def _set_res(fut, v):
        if not fut.done():
            fut.set_result(v)

    @staticmethod
    def _set_exc(fut, e):
        if not fut.done():
            fut.set_exception(e)

    def send_control(self, obj: Any) -> None:
        conn = self._connection()
        with self._send_lock:
            conn.send_bytes(P.pack_control(obj))

    def decode_answers(self, seqs: List[List[int]]) -> List[Dict[str, str]]:
        fields = self.fields
        return [null_rejection(dict(zip(fields, vals))) for vals in self.tok.decode_fields(seqs, len(fields))]

    def decode_response(self, buf: bytes) -> List[Dict[str, str]]:
        """Answers of one ``R`` frame (serving/protocol.py)."""
        fields = self.fields
        if self.fast is not None:
            n = P.count(buf)
            rows = self.fast.decode_fields(buf, P.HEADER_SIZE, n, len(fields))
        else:
            rows = self.tok.decode_fields(P.unpack_ids(buf)[2], len(fields))
        # a non-transaction (txn_type otp / unknown) comes back with null fields
        return [null_rejection(dict(zip(fields, vals))) for vals in rows]

    def decode_rows(self, buf: bytes) -> List[List[str]]:
        """The nine decoded field strings of every answer of one ``R`` frame, with no
        per-answer dict: the parser's native post-processing (parse/fastpath.py) reads
        them as they are (a non-transaction class is judged there)."""
        fields = self.fields
        if self.fast is not None:
            return self.fast.decode_fields(buf, P.HEADER_SIZE, P.count(buf), len(fields))
        return self.tok.decode_fields(P.unpack_ids(buf)[2], len(fields))

    def encode_request(self, rid: int, bodies: Sequence[str]) -> bytes:
        """The ``Q`` frame of ``bodies``: ``body <ans>`` ids, each body cut to max_body
        tokens (counted like ExtractorTokenizer.message_ids)."""
        if self.fast is None:
            return P.pack_ids(b"Q", rid, self.tok.message_ids(list(bodies), self.max_body))
        cut, lens, flat = self.fast.encode_packed(bodies, self.max_body, self.tok.ans)
        if cut:
            self.tok.truncated += cut
            from ..obs.metrics import LLM_TRUNCATED

            LLM_TRUNCATED.inc(cut)
        return P.pack_raw(b"Q", rid, len(bodies), lens, flat)

    async def extract(self, bodies: Sequence[str]) -> List[Dict[str, str]]:
        return self.decode_response(await self._roundtrip(bodies))

    async def extract_rows(self, bodies: Sequence[str]) -> List[List[str]]:
        """:meth:`extract` as answer rows (:meth:`decode_rows`)."""
        return self.decode_rows(await self._roundtrip(bodies))

    async def _roundtrip(self, bodies: Sequence[str]) -> bytes:
        rid = next(self._ids)
        msg = self.encode_request(rid, bodies)
        conn = self._connection()  # may raise BackendUnavailable: nothing registered yet
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._plock:
            self._pending[rid] = (fut, loop, conn)
        sent = False
        try:
            if self.conn is not conn:  # its reader already swept: it will never answer
                raise self._unavailable("engine server closed")
            with self._send_lock:
                conn.send_bytes(msg)
            sent = True
        except OSError as exc:  # broken pipe: the server went away under us
            with self._conn_lock:
                if self.conn is conn:
                    self.conn = None
            raise self._unavailable(f"engine server send failed: {exc}") from exc
        finally:
            if not sent:
                with self._plock:
                    self._pending.pop(rid, None)
        try:
            buf = await (asyncio.wait_for(fut, self.request_timeout) if self.request_timeout else fut)
        except asyncio.TimeoutError:
            with self._plock:
                self._pending.pop(rid, None)
            raise self._unavailable(f"engine server did not answer within {self.request_timeout:.0f} s") from None
        return buf
