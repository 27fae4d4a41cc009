"""Synchronous broker core: streams, retention, durable competing consumers.

One :class:`Engine` instance is the whole state machine of the bus. It is
single-threaded by design (the owning event loop or the broker process calls
it) and I/O free; persistence is layered on top through the ``journal``
callback (see :mod:`smsgate_amd.bus.filelog`), which receives every mutating
event so the state can be rebuilt by replay.

Costs are O(1) amortised per message per consumer: a consumer walks the
stream's sequence space once with a cursor, un-acked deliveries sit in a dict
plus a lazily-invalidated deadline heap, and ``num_pending`` is maintained
incrementally instead of being recounted (the reference polled
``consumer_info`` every 1-5 s, writer.py:46-54, worker.py:220-224).
"""
from __future__ import annotations

import heapq
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from .base import (
    BusError,
    BusUnavailable,
    ConsumerConfig,
    ConsumerInfo,
    DeliverPolicy,
    StreamConfig,
    StreamInfo,
    subject_matches,
)

__all__ = ["Engine", "Stored", "Delivery"]

Journal = Callable[[str, tuple], None]


@dataclass
class Stored:
    seq: int
    subject: str
    data: bytes
    ts: float
    headers: Optional[Dict[str, str]] = None


@dataclass
class Delivery:
    msg: Stored
    num_delivered: int


@dataclass
class _Consumer:
    cfg: ConsumerConfig
    cursor: int  # highest seq already considered for first delivery
    pending: Dict[int, List[float]] = field(default_factory=dict)  # seq -> [deadline, n_delivered]
    heap: List[Tuple[float, int]] = field(default_factory=list)  # (ready_at, seq), lazy
    num_pending: int = 0  # matching & stored & > cursor
    num_redelivered: int = 0
    num_dropped: int = 0

    def matches(self, subject: str, cache: Dict[Tuple[str, str], bool]) -> bool:
        key = (self.cfg.filter_subject, subject)
        hit = cache.get(key)
        if hit is None:
            hit = cache[key] = subject_matches(self.cfg.filter_subject, subject)
        return hit


class _Stream:
    def __init__(self, cfg: StreamConfig, first_seq: int = 1) -> None:
        self.cfg = cfg
        self.msgs: Dict[int, Stored] = {}
        self.first_seq = first_seq  # lowest seq possibly still stored
        self.last_seq = first_seq - 1
        self.bytes = 0
        self.consumers: Dict[str, _Consumer] = {}


class Engine:
    """In-memory state machine of a JetStream-like bus."""

    def __init__(self, journal: Optional[Journal] = None, clock: Callable[[], float] = time.time) -> None:
        self.streams: Dict[str, _Stream] = {}
        self._journal = journal
        self._clock = clock
        self._match_cache: Dict[Tuple[str, str], bool] = {}
        self._route_cache: Dict[str, Optional[_Stream]] = {}

    # ------------------------------------------------------------------ streams
    def _log(self, kind: str, *args) -> None:
        if self._journal is not None:
            self._journal(kind, args)

    def add_or_update_stream(self, cfg: StreamConfig) -> StreamInfo:
        st = self.streams.get(cfg.name)
        if st is None:
            for other in self.streams.values():
                for s in cfg.subjects:
                    if any(subject_matches(o, s) or subject_matches(s, o) for o in other.cfg.subjects):
                        raise BusError(f"subject {s!r} overlaps stream {other.cfg.name!r}")
            st = self.streams[cfg.name] = _Stream(cfg)
        else:
            st.cfg = cfg
        self._route_cache.clear()
        self._log("stream", cfg.name, list(cfg.subjects), cfg.max_age, cfg.max_msgs, cfg.max_bytes, cfg.storage)
        return self.stream_info(cfg.name)

    def _route(self, subject: str) -> _Stream:
        st = self._route_cache.get(subject, False)
        if st is False:
            st = None
            for cand in self.streams.values():
                if any(subject_matches(p, subject) for p in cand.cfg.subjects):
                    st = cand
                    break
            self._route_cache[subject] = st
        if st is None:  # every message to it would fail alike: not one message's fault
            raise BusUnavailable(f"no stream matches subject {subject!r}")
        return st

    def store(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None,
              ts: Optional[float] = None, seq: Optional[int] = None) -> Tuple[str, int]:
        st = self._route(subject)
        ts = self._clock() if ts is None else ts
        seq = st.last_seq + 1 if seq is None else seq
        st.last_seq = seq
        st.msgs[seq] = Stored(seq, subject, data, ts, headers)
        st.bytes += len(data)
        for c in st.consumers.values():
            if seq > c.cursor and c.matches(subject, self._match_cache):
                c.num_pending += 1
        self._log("store", st.cfg.name, seq, subject, data, ts, headers)
        self._enforce_limits(st)
        return st.cfg.name, seq

    def store_many(self, items, ts: Optional[float] = None) -> List[Tuple[str, int]]:
        """Batched :meth:`store` (one clock read, retention applied once per
        touched stream at the end — the same final state, since retention only
        ever drops from the front)."""
        ts = self._clock() if ts is None else ts
        route, log, mc = self._route, self._journal, self._match_cache
        out: List[Tuple[str, int]] = []
        touched: Dict[str, _Stream] = {}
        for subject, data in items:
            st = route(subject)
            seq = st.last_seq = st.last_seq + 1
            st.msgs[seq] = Stored(seq, subject, data, ts, None)
            st.bytes += len(data)
            for c in st.consumers.values():
                if seq > c.cursor and c.matches(subject, mc):
                    c.num_pending += 1
            name = st.cfg.name
            if log is not None:
                log("store", (name, seq, subject, data, ts, None))
            touched[name] = st
            out.append((name, seq))
        for st in touched.values():
            self._enforce_limits(st)
        return out

    def _drop(self, st: _Stream, seq: int) -> None:
        m = st.msgs.pop(seq, None)
        if m is None:
            return
        st.bytes -= len(m.data)
        for c in st.consumers.values():
            if seq > c.cursor:
                if c.matches(m.subject, self._match_cache):
                    c.num_pending -= 1
            else:
                c.pending.pop(seq, None)

    def _enforce_limits(self, st: _Stream) -> None:
        cfg = st.cfg
        while st.first_seq <= st.last_seq and st.first_seq not in st.msgs:
            st.first_seq += 1
        if cfg.max_msgs >= 0:
            while len(st.msgs) > cfg.max_msgs:
                self._drop(st, st.first_seq)
                st.first_seq += 1
        if cfg.max_bytes >= 0:
            while st.bytes > cfg.max_bytes and st.msgs:
                self._drop(st, st.first_seq)
                st.first_seq += 1
        while st.first_seq <= st.last_seq and st.first_seq not in st.msgs:
            st.first_seq += 1

    def expire(self, now: Optional[float] = None) -> int:
        """Apply ``max_age`` retention; returns the number of messages removed."""
        now = self._clock() if now is None else now
        n = 0
        for st in self.streams.values():
            if st.cfg.max_age <= 0:
                continue
            horizon = now - st.cfg.max_age
            while st.first_seq <= st.last_seq:
                m = st.msgs.get(st.first_seq)
                if m is not None:
                    if m.ts >= horizon:
                        break
                    self._drop(st, st.first_seq)
                    n += 1
                st.first_seq += 1
        return n

    def purge(self, stream: str) -> None:
        st = self._stream(stream)
        for seq in list(st.msgs):
            self._drop(st, seq)
        st.first_seq = st.last_seq + 1
        self._log("purge", stream)

    def _stream(self, name: str) -> _Stream:
        st = self.streams.get(name)
        if st is None:
            raise BusError(f"stream {name!r} not found")
        return st

    def stream_info(self, name: str) -> StreamInfo:
        st = self._stream(name)
        return StreamInfo(
            config=st.cfg,
            messages=len(st.msgs),
            bytes=st.bytes,
            first_seq=st.first_seq,
            last_seq=st.last_seq,
            consumers=len(st.consumers),
        )

    def stream_for_subject(self, subject: str) -> str:
        return self._route(subject).cfg.name

    # ---------------------------------------------------------------- consumers
    def add_consumer(self, stream: str, cfg: ConsumerConfig) -> ConsumerInfo:
        st = self._stream(stream)
        c = st.consumers.get(cfg.durable)
        if c is None:
            if cfg.deliver_policy == DeliverPolicy.ALL:
                cursor = st.first_seq - 1
            elif cfg.deliver_policy == DeliverPolicy.NEW:
                cursor = st.last_seq
            else:  # LAST: deliver the newest matching message and everything after
                cursor = st.last_seq
                for seq in range(st.last_seq, st.first_seq - 1, -1):
                    m = st.msgs.get(seq)
                    if m is not None and subject_matches(cfg.filter_subject, m.subject):
                        cursor = seq - 1
                        break
            c = _Consumer(cfg=cfg, cursor=cursor)
            c.num_pending = sum(
                1 for s, m in st.msgs.items() if s > cursor and c.matches(m.subject, self._match_cache)
            )
            st.consumers[cfg.durable] = c
        else:
            # Rebinding keeps the durable position; allow tuning of timers/limits.
            old = c.cfg
            c.cfg = ConsumerConfig(
                durable=cfg.durable,
                filter_subject=old.filter_subject,
                ack_wait=cfg.ack_wait,
                max_deliver=cfg.max_deliver,
                deliver_policy=old.deliver_policy,
                max_ack_pending=cfg.max_ack_pending,
            )
            if cfg.filter_subject != old.filter_subject:
                raise BusError(
                    f"durable {cfg.durable!r} is bound to {old.filter_subject!r}, not {cfg.filter_subject!r}"
                )
        self._log("consumer", stream, cfg.durable, cfg.filter_subject, cfg.ack_wait, cfg.max_deliver,
                  cfg.deliver_policy.value, cfg.max_ack_pending, c.cursor)
        return self.consumer_info(stream, cfg.durable)

    def delete_consumer(self, stream: str, durable: str) -> None:
        self._stream(stream).consumers.pop(durable, None)
        self._log("delconsumer", stream, durable)

    def _consumer(self, stream: str, durable: str) -> Tuple[_Stream, _Consumer]:
        st = self._stream(stream)
        c = st.consumers.get(durable)
        if c is None:
            raise BusError(f"consumer {durable!r} not found on stream {stream!r}")
        return st, c

    def next_batch(self, stream: str, durable: str, n: int, now: Optional[float] = None) -> List[Delivery]:
        """Hand out up to ``n`` messages: due redeliveries first, then new ones."""
        now = self._clock() if now is None else now
        st, c = self._consumer(stream, durable)
        out: List[Delivery] = []
        heap = c.heap
        # 1) redeliveries whose ack-wait (or nak delay) elapsed
        while heap and len(out) < n and heap[0][0] <= now:
            ready, seq = heapq.heappop(heap)
            ent = c.pending.get(seq)
            if ent is None or ent[0] != ready:
                continue  # stale heap entry (acked, or re-armed)
            m = st.msgs.get(seq)
            if m is None:
                c.pending.pop(seq, None)
                continue
            if 0 < c.cfg.max_deliver <= ent[1]:
                c.pending.pop(seq, None)
                c.num_dropped += 1
                self._log("term", stream, durable, seq)
                continue
            ent[1] += 1
            ent[0] = now + c.cfg.ack_wait
            heapq.heappush(heap, (ent[0], seq))
            c.num_redelivered += 1
            out.append(Delivery(m, int(ent[1])))
        # 2) first deliveries past the cursor
        room = c.cfg.max_ack_pending - len(c.pending)
        start = c.cursor
        while len(out) < n and room > 0 and c.cursor < st.last_seq:
            c.cursor += 1
            m = st.msgs.get(c.cursor)
            if m is None or not c.matches(m.subject, self._match_cache):
                continue
            c.num_pending -= 1
            deadline = now + c.cfg.ack_wait
            c.pending[m.seq] = [deadline, 1]
            heapq.heappush(heap, (deadline, m.seq))
            out.append(Delivery(m, 1))
            room -= 1
        if c.cursor != start:
            self._log("cursor", stream, durable, c.cursor)
        return out

    def ack(self, stream: str, durable: str, seq: int) -> bool:
        _, c = self._consumer(stream, durable)
        hit = c.pending.pop(seq, None) is not None
        if hit:
            self._log("ack", stream, durable, seq)
        return hit

    def term(self, stream: str, durable: str, seq: int) -> bool:
        _, c = self._consumer(stream, durable)
        hit = c.pending.pop(seq, None) is not None
        if hit:
            c.num_dropped += 1
            self._log("term", stream, durable, seq)
        return hit

    def nak(self, stream: str, durable: str, seq: int, delay: float = 0.0,
            now: Optional[float] = None) -> bool:
        now = self._clock() if now is None else now
        _, c = self._consumer(stream, durable)
        ent = c.pending.get(seq)
        if ent is None:
            return False
        ent[0] = now + max(0.0, delay)
        heapq.heappush(c.heap, (ent[0], seq))
        return True

    def touch(self, stream: str, durable: str, seq: int, now: Optional[float] = None) -> bool:
        now = self._clock() if now is None else now
        _, c = self._consumer(stream, durable)
        ent = c.pending.get(seq)
        if ent is None:
            return False
        ent[0] = now + c.cfg.ack_wait
        heapq.heappush(c.heap, (ent[0], seq))
        return True

    def next_ready_at(self, stream: str, durable: str) -> Optional[float]:
        """Earliest time a pending message becomes re-deliverable (None = none)."""
        _, c = self._consumer(stream, durable)
        heap = c.heap
        while heap:
            ready, seq = heap[0]
            ent = c.pending.get(seq)
            if ent is None or ent[0] != ready:
                heapq.heappop(heap)
                continue
            return ready
        return None

    def has_new(self, stream: str, durable: str) -> bool:
        st, c = self._consumer(stream, durable)
        return c.num_pending > 0 and len(c.pending) < c.cfg.max_ack_pending

    def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        _, c = self._consumer(stream, durable)
        floor = (min(c.pending) - 1) if c.pending else c.cursor
        return ConsumerInfo(
            stream=stream,
            name=durable,
            num_pending=c.num_pending,
            num_ack_pending=len(c.pending),
            num_redelivered=c.num_redelivered,
            delivered_seq=c.cursor,
            ack_floor=floor,
        )

    # --------------------------------------------------------------- snapshot
    def snapshot(self) -> dict:
        """A JSON-able image of the whole state (used for log compaction)."""
        out = {"streams": []}
        for st in self.streams.values():
            out["streams"].append(
                {
                    "cfg": [st.cfg.name, list(st.cfg.subjects), st.cfg.max_age, st.cfg.max_msgs,
                            st.cfg.max_bytes, st.cfg.storage],
                    "first_seq": st.first_seq,
                    "last_seq": st.last_seq,
                    "consumers": [
                        {
                            "cfg": [c.cfg.durable, c.cfg.filter_subject, c.cfg.ack_wait, c.cfg.max_deliver,
                                    c.cfg.deliver_policy.value, c.cfg.max_ack_pending],
                            "cursor": c.cursor,
                            "pending": {str(k): v[1] for k, v in c.pending.items()},
                            "redelivered": c.num_redelivered,
                        }
                        for c in st.consumers.values()
                    ],
                }
            )
        return out
