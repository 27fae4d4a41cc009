"""Crash-safe persistence for the bus engine: an append-only framed journal.

The reference delegates durability to the NATS server's file store
(``-js -sd=/data``, docker-compose.yml:19-27): streams survive restarts and
durable consumers resume from their last ack.  Here the
in-memory :class:`~smsgate_amd.bus.engine.Engine` emits every mutating event
through its ``journal`` hook; :class:`FileLog` appends them to segment files

    ``<dir>/journal-<n>.log``: [u32 length][u32 crc32][msgpack (kind, args)] ...

and recovery replays them into a fresh engine.  Delivered-but-unacked
messages at crash time become pending again and are redelivered at once
(at-least-once).  When the live journal exceeds ``compact_bytes`` the state is
rewritten as one compact segment (streams, consumers, cursors, pending sets,
stored messages) and older segments are deleted.  A torn tail frame (crash in
mid-write) is detected by length/CRC and truncated.

``fsync`` policy: ``"always"`` (every event), ``"interval"`` (default: flush
each event to the OS, fsync at most every ``fsync_interval_s``), ``"never"``.
"""
from __future__ import annotations

import os
import struct
import threading
import time
import zlib
from pathlib import Path
from typing import Any, Iterator, List, Optional, Tuple

import msgpack

from .base import ConsumerConfig, DeliverPolicy, StreamConfig
from .engine import Engine

__all__ = ["FileLog", "open_file_bus", "replay_into"]

_FRAME = struct.Struct("<II")


def _frames(path: Path) -> Iterator[Tuple[int, Any]]:
    """Yield (end_offset, record) for every intact frame; stops at a torn tail."""
    with open(path, "rb") as f:
        data = f.read()
    off = 0
    n = len(data)
    while off + _FRAME.size <= n:
        ln, crc = _FRAME.unpack_from(data, off)
        end = off + _FRAME.size + ln
        if end > n:
            break
        body = data[off + _FRAME.size:end]
        if zlib.crc32(body) != crc:
            break
        yield end, msgpack.unpackb(body, raw=False, strict_map_key=False)
        off = end


def replay_into(eng: Engine, kind: str, args: list) -> None:
    """Apply one journal event to an engine whose own journal is disabled."""
    if kind == "stream":
        name, subjects, max_age, max_msgs, max_bytes, storage = args
        eng.add_or_update_stream(StreamConfig(name, list(subjects), max_age, max_msgs, max_bytes, storage))
    elif kind == "store":
        stream, seq, subject, data, ts, headers = args
        st = eng.streams[stream]
        if seq > st.last_seq:
            eng.store(subject, data, headers, ts=ts, seq=seq)
    elif kind == "consumer":
        stream, durable, filt, ack_wait, max_deliver, policy, max_ack_pending, cursor = args
        st = eng.streams[stream]
        if durable not in st.consumers:
            eng.add_consumer(stream, ConsumerConfig(durable, filt, ack_wait, max_deliver, DeliverPolicy(policy),
                                                    max_ack_pending))
            st.consumers[durable].cursor = cursor
            _recount(eng, stream, durable)
        else:
            c = st.consumers[durable]
            c.cfg = ConsumerConfig(durable, filt, ack_wait, max_deliver, DeliverPolicy(policy), max_ack_pending)
    elif kind == "cursor":
        stream, durable, new = args
        st = eng.streams[stream]
        c = st.consumers.get(durable)
        if c is None:
            return
        for seq in range(c.cursor + 1, new + 1):
            m = st.msgs.get(seq)
            if m is not None and c.matches(m.subject, eng._match_cache):
                c.pending[seq] = [0.0, 1]  # delivered before the crash: redeliver at once
                c.num_pending -= 1
        c.cursor = max(c.cursor, new)
    elif kind in ("ack", "term"):
        stream, durable, seq = args
        c = eng.streams[stream].consumers.get(durable)
        if c is not None:
            c.pending.pop(seq, None)
    elif kind == "delconsumer":
        stream, durable = args
        eng.streams[stream].consumers.pop(durable, None)
    elif kind == "purge":
        eng.purge(args[0])
    elif kind == "pending":  # compacted snapshot of a consumer's unacked set
        stream, durable, seqs = args
        c = eng.streams[stream].consumers.get(durable)
        if c is not None:
            for s in seqs:
                if s in eng.streams[stream].msgs:
                    c.pending[int(s)] = [0.0, 1]


def _recount(eng: Engine, stream: str, durable: str) -> None:
    st = eng.streams[stream]
    c = st.consumers[durable]
    c.num_pending = sum(1 for s, m in st.msgs.items() if s > c.cursor and c.matches(m.subject, eng._match_cache))


class FileLog:
    def __init__(self, directory: str | os.PathLike, *, fsync: str = "interval", fsync_interval_s: float = 0.05,
                 compact_bytes: int = 256 << 20) -> None:
        self.dir = Path(directory)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.fsync = fsync
        self.fsync_interval_s = fsync_interval_s
        self.compact_bytes = compact_bytes
        self._lock = threading.Lock()
        self._f = None
        self._seg = 0
        self._bytes = 0
        self._floor_bytes = 0
        self._last_sync = time.monotonic()
        self.engine: Optional[Engine] = None
        self._need_compact = False

    # ------------------------------------------------------------------ files
    def _segments(self) -> List[Path]:
        return sorted(self.dir.glob("journal-*.log"))

    def _open_segment(self, n: int) -> None:
        if self._f is not None:
            self._f.flush()
            os.fsync(self._f.fileno())
            self._f.close()
        self._seg = n
        self._f = open(self.dir / f"journal-{n:08d}.log", "ab")
        self._bytes = self._f.tell()
        self._floor_bytes = self._bytes  # size right after a snapshot / at recovery

    def _write(self, kind: str, args) -> None:
        body = msgpack.packb([kind, list(args)], use_bin_type=True)
        frame = _FRAME.pack(len(body), zlib.crc32(body)) + body
        with self._lock:
            self._f.write(frame)
            self._bytes += len(frame)
            if self.fsync == "always":
                self._f.flush()
                os.fsync(self._f.fileno())
            elif self.fsync == "interval":
                self._f.flush()
                now = time.monotonic()
                if now - self._last_sync >= self.fsync_interval_s:
                    os.fsync(self._f.fileno())
                    self._last_sync = now
        # compact between operations, never mid-mutation; and only once the journal has
        # doubled since the last snapshot (a live state above compact_bytes would
        # otherwise be rewritten after every single append)
        if self._bytes > max(self.compact_bytes, 2 * self._floor_bytes):
            self._need_compact = True

    def maybe_compact(self) -> None:
        if self._need_compact:
            self._need_compact = False
            self.compact()

    # --------------------------------------------------------------- recovery
    def open(self) -> Engine:
        eng = Engine()
        segs = self._segments()
        for seg in segs:
            good_end = 0
            for end, (kind, args) in _frames(seg):
                replay_into(eng, kind, args)
                good_end = end
            if seg.stat().st_size != good_end:  # torn tail: drop it
                with open(seg, "r+b") as f:
                    f.truncate(good_end)
        import heapq

        for st in eng.streams.values():
            for d, con in st.consumers.items():
                _recount(eng, st.cfg.name, d)
                con.heap = [(v[0], s) for s, v in con.pending.items()]  # redeliver unacked at once
                heapq.heapify(con.heap)
        self._open_segment((int(segs[-1].stem.split("-")[1]) if segs else 0) + (0 if segs else 1))
        eng._journal = self._write
        self.engine = eng
        return eng

    def compact(self) -> None:
        """Rewrite the whole state as one fresh segment, then drop older ones."""
        eng = self.engine
        if eng is None:
            return
        old = self._segments()
        n = self._seg + 1
        tmp = self.dir / f"journal-{n:08d}.log.tmp"
        with open(tmp, "wb") as f:
            def put(kind, args):
                body = msgpack.packb([kind, list(args)], use_bin_type=True)
                f.write(_FRAME.pack(len(body), zlib.crc32(body)) + body)

            for st in eng.streams.values():
                c = st.cfg
                put("stream", (c.name, c.subjects, c.max_age, c.max_msgs, c.max_bytes, c.storage))
                for seq in sorted(st.msgs):
                    m = st.msgs[seq]
                    put("store", (c.name, m.seq, m.subject, m.data, m.ts, m.headers))
                for d, con in st.consumers.items():
                    cc = con.cfg
                    put("consumer", (c.name, d, cc.filter_subject, cc.ack_wait, cc.max_deliver,
                                     cc.deliver_policy.value, cc.max_ack_pending, con.cursor))
                    put("pending", (c.name, d, sorted(con.pending)))
            f.flush()
            os.fsync(f.fileno())
        with self._lock:
            final = self.dir / f"journal-{n:08d}.log"
            os.replace(tmp, final)
            self._open_segment(n)
            for p in old:
                if p != final:
                    p.unlink(missing_ok=True)

    def close(self) -> None:
        with self._lock:
            if self._f is not None:
                self._f.flush()
                os.fsync(self._f.fileno())
                self._f.close()
                self._f = None


async def open_file_bus(directory: str, max_age: float = 3 * 24 * 3600.0, **kw):
    """``file://`` DSN: an in-process :class:`MemoryBus` over a journaled engine."""
    from .base import default_stream_config
    from .memory import MemoryBus

    log = FileLog(directory, **kw)
    eng = log.open()
    bus = MemoryBus(eng, create_default_stream=False)
    if not eng.streams:
        eng.add_or_update_stream(default_stream_config(max_age))
    bus._filelog = log  # type: ignore[attr-defined]
    orig_close = bus.close

    async def close() -> None:
        await orig_close()
        log.close()

    bus.close = close  # type: ignore[method-assign]
    pub, pub_many = bus.publish, bus.publish_many

    async def publish(*a, **k):
        r = await pub(*a, **k)
        log.maybe_compact()
        return r

    async def publish_many(*a, **k):
        r = await pub_many(*a, **k)
        log.maybe_compact()
        return r

    bus.publish, bus.publish_many = publish, publish_many  # type: ignore[method-assign]
    return bus
