"""Subject-sharded bus: several brokers act as one bus, each owning some subjects.

The reference runs ONE NATS server for everything (docker-compose.yml:15-27).
One ``smsgate-busd`` event loop carries ≈250 k publish→fetch→ack messages/s with
its journal on (tests/test_broker_capacity.py), while a node of 8 GPUs needs
about one message per SMS on each of three subjects at ~25 k SMS/s per GPU.
Sharding by subject keeps every subject's semantics intact (one stream per
broker, one competing consumer group per durable, a durable lives where its
subject lives) and splits the broker work.

Two layouts, chosen by the DSN:

* **positional** (``sharded+A,B,C``): ``sms.raw`` on shard 0; with two shards
  the parser's outputs (``sms.parsed`` / ``sms.processing`` / ``sms.failed`` /
  ``sms.categorized``) on shard 1; with three (the 8-GPU deployment) one message
  per SMS lands on each shard: sms.parsed alone on 1, sms.processing (and the
  low-rate subjects) on 2 (:func:`shard_of`);
* **pinned** (``sharded+sms.raw=A,sms.raw=B,sms.parsed=C,*=D``): a member
  prefixed ``<subject>=`` serves that subject, and a subject pinned to several
  members is **partitioned** over them: publishes are dealt round-robin, a
  durable exists on every partition (one competing group per partition, the
  same name), and a subscription fetches from the partitions in rotation, so
  a subject's rate is no longer bounded by one broker's event loop.  Unpinned
  subjects go to the ``*=`` (or unprefixed) members, spread by subject hash.

``consumer_info`` of a partitioned durable sums its partitions.
"""
from __future__ import annotations

import asyncio
from collections.abc import Sequence as SequenceABC
import time
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

from .base import (
    SUBJECT_PARSED,
    SUBJECT_PROCESSING,
    SUBJECT_RAW,
    Bus,
    BusError,
    BusUnavailable,
    ConsumerInfo,
    Msg,
    PubAck,
    StreamConfig,
    StreamInfo,
    Subscription,
)

__all__ = ["ShardedBus", "shard_of", "parse_members", "Router", "NODE_PARTITIONS", "node_layout", "node_partitions"]

# The 8-GPU node's broker layout (deploy/docker-compose.yml is generated from it by
# deploy/gen_compose.py; bench.py): every per-SMS subject partitioned -- sms.raw (one
# publish + delivery + ack per SMS) over twenty brokers, each also a native HTTP ingest
# door (smsgate-busd --http-listen: ~56 k single-SMS requests/s each,
# profiles/r03_ingest_bench.jsonl: 20 doors take 2x an 8 x 70 k node), sms.parsed
# (parser -> writer) and sms.processing (one publish per parsed SMS, consumed
# downstream) over six each (a member carries ~0.9 / 6 of the node rate, 83 k msgs/s at
# an 8 x 69.5 k node: 2x headroom on one broker down to 167 k msgs/s -- the
# 16-consumer load generator measured 204-248 k with the journal on disk on a busy
# 8-vCPU build box, 316 k on a quiet one; four partitions needed 250 k) -- and the
# low-rate subjects (sms.failed, sms.categorized) on one more.
# tests/test_broker_capacity.py sizes EVERY member and the doors at 2x against the
# latest measured headline.  Fewer GPUs on a node:
# node_partitions() scales it down.
NODE_PARTITIONS = {SUBJECT_RAW: 20, SUBJECT_PARSED: 6, SUBJECT_PROCESSING: 6}
NODE_GPUS = 8


def node_partitions(gpus: int = NODE_GPUS) -> Dict[str, int]:
    """The node layout sized for ``gpus`` GPUs (same per-broker load as the 8-GPU node)."""
    return {s: max(1, -(-n * gpus // NODE_GPUS)) for s, n in NODE_PARTITIONS.items()}


def node_layout(dsns: Sequence[str], partitions: Optional[Dict[str, int]] = None) -> str:
    """Pinned ``sharded+`` DSN over ``dsns``: the first ``partitions[s]`` members per
    subject (in dict order), the remaining member(s) as the default."""
    parts = NODE_PARTITIONS if partitions is None else partitions
    need = sum(parts.values()) + 1
    if len(dsns) < need:
        raise BusError(f"layout {parts} needs {need} brokers, got {len(dsns)}")
    out, k = [], 0
    for subject, n in parts.items():
        for _ in range(n):
            out.append(f"{subject}={dsns[k]}")
            k += 1
    out += [f"*={d}" for d in dsns[k:]]
    return "sharded+" + ",".join(out)


def shard_of(subject: str, n: int) -> int:
    """Positional layout: shard owning ``subject``: ingest (sms.raw) on 0; with 3+
    shards sms.parsed alone on 1, sms.processing on 2 and the rest spread over 2 .. n-1."""
    if n <= 1 or subject == SUBJECT_RAW:
        return 0
    if n == 2 or subject == SUBJECT_PARSED:
        return 1
    if subject == SUBJECT_PROCESSING:
        return 2
    return 2 + zlib.crc32(subject.encode()) % (n - 2)


def parse_members(spec: str) -> Tuple[List[str], Dict[str, List[int]], List[int]]:
    """``"sms.raw=unix:///a,*=unix:///b"`` -> (member dsns, {subject: member indices},
    default member indices).  No ``=`` prefix anywhere -> positional layout ({} pins)."""
    dsns: List[str] = []
    pins: Dict[str, List[int]] = {}
    default: List[int] = []
    parts = [p for p in spec.split(",") if p]
    pinned = any("=" in p.split("://", 1)[0] for p in parts)
    for p in parts:
        head = p.split("://", 1)[0]
        if pinned and "=" in head:
            subj, dsn = p.split("=", 1)
        else:
            subj, dsn = "*", p
        idx = len(dsns)
        dsns.append(dsn)
        if subj == "*":
            default.append(idx)
        else:
            pins.setdefault(subj, []).append(idx)
    if pinned and not default:
        raise BusError(f"sharded DSN {spec!r}: pinned layout needs a '*=' member for the other subjects")
    return dsns, pins, default


class Router:
    """Subject -> member indices (one member, or the partitions of a pinned subject)."""

    def __init__(self, n: int, pins: Optional[Dict[str, List[int]]] = None,
                 default: Optional[List[int]] = None) -> None:
        self.n = n
        self.pins = dict(pins or {})
        self.default = list(default or range(n))
        # one dealing counter PER subject: a shared one would put every sms.parsed publish
        # on the even turns and every sms.processing one on the odd turns of a parser
        # batch that publishes them in pairs -- one partition of each would get nothing
        self._rr: Dict[str, int] = {}  # per partitioned subject: messages dealt so far

    def members(self, subject: str) -> List[int]:
        if not self.pins:
            return [shard_of(subject, self.n)]
        if subject in self.pins:
            return self.pins[subject]
        return [self.default[zlib.crc32(subject.encode()) % len(self.default)]]

    def publish_target(self, subject: str) -> int:
        ms = self.members(subject)
        if len(ms) == 1:
            return ms[0]
        k = self._rr.get(subject, 0)
        self._rr[subject] = k + 1
        return ms[k % len(ms)]

    def deal(self, subject: str, n: int) -> List[Tuple[int, slice]]:
        """``n`` messages of ``subject`` dealt round-robin over its members, exactly as
        ``n`` calls of :meth:`publish_target` would: ``(member, slice of the n)`` pairs."""
        ms = self.members(subject)
        if len(ms) == 1:
            return [(ms[0], slice(0, n))]
        k = self._rr.get(subject, 0)
        self._rr[subject] = k + n
        m = len(ms)
        return [(ms[(k + r) % m], slice(r, n, m)) for r in range(min(m, n))]


class _MergedAcks(SequenceABC):
    """publish_many's acks in publish order, gathered from the members' replies only
    when read (the hot publishers never read them)."""

    __slots__ = ("_n", "_parts", "_flat")

    def __init__(self, n: int, parts) -> None:
        self._n, self._parts, self._flat = n, parts, None

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if self._flat is None:
            flat: List[Optional[PubAck]] = [None] * self._n
            for idx, acks in self._parts:
                for k, a in zip(idx, acks):
                    flat[k] = a
            self._flat = flat
        return self._flat[i]

    def __eq__(self, other) -> bool:
        if not isinstance(other, SequenceABC):
            return NotImplemented
        return list(self) == list(other)


class _PartitionedSub(Subscription):
    """One durable on every partition of a subject.

    ``fetch`` first sweeps the partitions without waiting (rotating the start so
    no partition starves), then long-polls EVERY partition at once and returns as
    soon as one answers.  A long-poll still outstanding when the call returns is
    kept, never cancelled: whatever it delivers later is buffered and returned by
    the next ``fetch`` (cancelling it would strand the messages it was handed
    until ack_wait).  So at low load a message on any partition is picked up
    immediately, not after ``(n-1)`` polling slices.

    A partition whose fetch raises (its broker is down) is skipped with an
    exponential backoff (``BACKOFF_MIN``..``BACKOFF_MAX``) while the healthy ones
    keep being served; messages already pulled in the same call are returned,
    not dropped.  ``fetch`` raises only when every partition is failing."""

    BACKOFF_MIN = 0.05
    BACKOFF_MAX = 2.0
    LONG_POLL = 1.0  # seconds one background long-poll may stay outstanding

    def __init__(self, subs: Sequence[Subscription]) -> None:
        self.subs = list(subs)
        self.consumer = subs[0].consumer
        self.stream = getattr(subs[0], "stream", None) or "SMS"
        self._rr = 0
        n = len(self.subs)
        self._down_until = [0.0] * n
        self._backoff = [0.0] * n
        self._inflight: Dict[int, "asyncio.Task[List[Msg]]"] = {}
        self._buffer: List[Msg] = []
        self.partition_errors = 0
        self._last_error: Optional[BaseException] = None

    def _failed(self, i: int, exc: BaseException) -> None:
        self.partition_errors += 1
        self._backoff[i] = min(self.BACKOFF_MAX, max(self.BACKOFF_MIN, self._backoff[i] * 2))
        self._down_until[i] = time.monotonic() + self._backoff[i]
        self._last_error = exc

    def _ok(self, i: int) -> None:
        self._backoff[i] = 0.0

    def _harvest(self, i: int, task: "asyncio.Task[List[Msg]]") -> List[Msg]:
        """Result of partition ``i``'s finished long-poll (it is removed from the
        in-flight set by exactly one caller)."""
        if self._inflight.get(i) is not task:
            return []
        del self._inflight[i]
        try:
            got = task.result()
        except asyncio.CancelledError:
            return []
        except Exception as exc:  # noqa: BLE001
            self._failed(i, exc)
            return []
        self._ok(i)
        return got

    def _take(self, got: List[Msg], batch: int) -> List[Msg]:
        if len(got) > batch:
            self._buffer = got[batch:] + self._buffer
            got = got[:batch]
        return got

    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        n = len(self.subs)
        start = self._rr
        self._rr = (self._rr + 1) % n
        got, self._buffer = self._buffer[:batch], self._buffer[batch:]
        for i, t in list(self._inflight.items()):
            if t.done():
                got += self._harvest(i, t)
        now = time.monotonic()
        order = [(start + k) % n for k in range(n)]
        live = [i for i in order if self._down_until[i] <= now]
        if not live and not self._inflight and not got:
            raise BusUnavailable(f"every partition of {self.consumer!r} is failing: {self._last_error}")
        for i in live:
            if len(got) >= batch:
                return self._take(got, batch)
            if i in self._inflight:
                continue
            try:
                got += await self.subs[i].fetch(batch - len(got), 0)
                self._ok(i)
            except Exception as exc:  # noqa: BLE001 - one broker down must not stall the others
                self._failed(i, exc)
        if got or (timeout is not None and timeout <= 0):
            return self._take(got, batch)
        now = time.monotonic()
        deadline = None if timeout is None else now + timeout
        for i in order:
            if i not in self._inflight and self._down_until[i] <= now:
                self._inflight[i] = asyncio.ensure_future(self.subs[i].fetch(batch, self.LONG_POLL))
        if not self._inflight:  # every partition is backing off: wait out the shortest backoff
            wait = min(self._down_until) - now
            await asyncio.sleep(max(0.0, min(wait, timeout if timeout is not None else wait)))
            return []
        while True:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            done, _ = await asyncio.wait(list(self._inflight.values()), timeout=left,
                                         return_when=asyncio.FIRST_COMPLETED)
            for i, t in list(self._inflight.items()):
                if t in done:
                    got += self._harvest(i, t)
            if got or not done or (deadline is not None and time.monotonic() >= deadline):
                return self._take(got, batch)
            # an empty long-poll ended (its own timeout): re-arm it and keep waiting
            now = time.monotonic()
            for i in order:
                if i not in self._inflight and self._down_until[i] <= now:
                    self._inflight[i] = asyncio.ensure_future(self.subs[i].fetch(batch, self.LONG_POLL))
            if not self._inflight:
                return []

    async def unsubscribe(self) -> None:
        for t in self._inflight.values():
            t.cancel()
        self._inflight.clear()
        await asyncio.gather(*(s.unsubscribe() for s in self.subs))


def _sum_infos(infos: Sequence[ConsumerInfo]) -> ConsumerInfo:
    first = infos[0]
    if len(infos) == 1:
        return first
    return ConsumerInfo(stream=first.stream, name=first.name,
                        num_pending=sum(i.num_pending for i in infos),
                        num_ack_pending=sum(i.num_ack_pending for i in infos),
                        num_redelivered=sum(i.num_redelivered for i in infos),
                        delivered_seq=max(i.delivered_seq for i in infos),
                        ack_floor=min(i.ack_floor for i in infos),
                        num_waiting=sum(i.num_waiting for i in infos))


class ShardedBus(Bus):
    def __init__(self, members: Sequence[Bus], pins: Optional[Dict[str, List[int]]] = None,
                 default: Optional[List[int]] = None) -> None:
        if not members:
            raise BusError("sharded bus needs at least one member")
        self.members = list(members)
        self.router = Router(len(self.members), pins, default)
        self._durables: Dict[Tuple[str, str], List[int]] = {}  # (stream, durable) -> shards

    @classmethod
    async def connect(cls, spec: Sequence[str] | str, max_age: float) -> "ShardedBus":
        from . import _open

        dsns, pins, default = parse_members(spec if isinstance(spec, str) else ",".join(spec))
        return cls([await _open(d, max_age) for d in dsns], pins, default)

    def _bus(self, subject: str) -> Bus:
        return self.members[self.router.publish_target(subject)]

    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo:
        infos = await asyncio.gather(*(m.ensure_stream(config) for m in self.members))
        return infos[0]

    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck:
        return await self._bus(subject).publish(subject, data, headers)

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        by_subject: Dict[str, List[int]] = {}
        for i, it in enumerate(items):
            by_subject.setdefault(it[0], []).append(i)
        groups: Dict[int, List[int]] = {}
        for subject, idx in by_subject.items():  # the per-message deal, one subject at a time
            for k, sl in self.router.deal(subject, len(idx)):
                groups.setdefault(k, []).extend(idx[sl])
        if len(by_subject) > 1:
            for g in groups.values():
                g.sort()  # each member receives its messages in publish order
        if len(groups) == 1:
            (k, _), = groups.items()
            return await self.members[k].publish_many(items)
        res = await asyncio.gather(*(self.members[k].publish_many([items[i] for i in idx])
                                     for k, idx in groups.items()))
        return _MergedAcks(len(items), list(zip(groups.values(), res)))

    async def subscribe(self, subject: str, durable: str, **consumer_opts) -> Subscription:
        ks = self.router.members(subject)
        subs = [await self.members[k].subscribe(subject, durable, **consumer_opts) for k in ks]
        self._durables[(getattr(subs[0], "stream", None) or "SMS", durable)] = ks
        return subs[0] if len(subs) == 1 else _PartitionedSub(subs)

    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo:
        ks = self._durables.get((stream, durable))
        if ks is not None:
            return _sum_infos([await self.members[k].consumer_info(stream, durable) for k in ks])
        found = []
        for m in self.members:  # a durable created by another client: find its shard(s)
            try:
                found.append(await m.consumer_info(stream, durable))
            except Exception:  # noqa: BLE001 — not on this shard
                continue
        if not found:
            raise BusError(f"consumer {durable!r} not found on any shard")
        return _sum_infos(found)

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
