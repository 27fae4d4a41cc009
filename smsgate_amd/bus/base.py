"""Transport-agnostic durable pub/sub contract.

The reference talks to NATS JetStream (libs/nats_utils.py):
one stream ``SMS`` over five subjects, file storage, LIMITS retention with a
3-day ``max_age``, durable consumers with explicit ack and server-default
ack-wait redelivery, and ``consumer_info`` stats (``num_pending``,
``num_ack_pending``).  This module defines the same semantics as an abstract
:class:`Bus` with three implementations:

* :class:`smsgate_amd.bus.memory.MemoryBus` — in-process (tests, benchmarks,
  single-process deployments);
* :class:`smsgate_amd.bus.server.BusServer` + :class:`smsgate_amd.bus.client.RemoteBus`
  — a broker process with a crash-safe segment log (``smsgate_amd.bus.filelog``)
  that any number of service processes reach over TCP/UDS;
* ``nats://`` DSNs map to an optional NATS adapter when ``nats-py`` exists.

Semantics (all backends):

* every consumer is *durable* and *competing*: each stored message matching
  its filter is handed to exactly one of the subscribers bound to that durable
  name (the reference's intended ``--group`` scaling, worker.py:199-202, which
  nats-py push consumers did not actually provide — SURVEY.md §2.10);
* delivery is at-least-once: a message not acked within ``ack_wait`` is
  redelivered; ``nak`` redelivers now (or after a delay); ``term`` drops it;
  ``max_deliver`` bounds attempts (``-1`` = unbounded);
* ``ensure_stream`` *creates* a missing stream (fixes D3) and updates subjects.
"""
from __future__ import annotations

import abc
import enum
import re
import time
from dataclasses import dataclass
from typing import AsyncIterator, Dict, List, Optional, Sequence, Tuple

__all__ = [
    "SUBJECT_RAW",
    "SUBJECT_PARSED",
    "SUBJECT_PROCESSING",
    "SUBJECT_FAILED",
    "SUBJECT_CATEGORIZED",
    "SUBJECT_FAILED_FINAL",
    "STREAM_NAME",
    "ALL_SUBJECTS",
    "DeliverPolicy",
    "StreamConfig",
    "ConsumerConfig",
    "PubAck",
    "StreamInfo",
    "ConsumerInfo",
    "Msg",
    "MsgMetadata",
    "Acker",
    "Subscription",
    "Bus",
    "BusError",
    "bus_error",
    "subject_matches",
    "default_stream_config",
]

# Subjects and stream of the reference (nats_utils.py:25-29, :64).
SUBJECT_RAW = "sms.raw"
SUBJECT_PARSED = "sms.parsed"
SUBJECT_PROCESSING = "sms.processing"
SUBJECT_FAILED = "sms.failed"
SUBJECT_CATEGORIZED = "sms.categorized"
# terminal DLQ: messages whose DLQ reparse failed again (no consumer in the pipeline:
# kept for inspection, never re-fed to the DLQ worker that reads sms.failed)
SUBJECT_FAILED_FINAL = "sms.failed.final"
STREAM_NAME = "SMS"
ALL_SUBJECTS = (SUBJECT_RAW, SUBJECT_PARSED, SUBJECT_FAILED, SUBJECT_PROCESSING, SUBJECT_CATEGORIZED,
                SUBJECT_FAILED_FINAL)


class BusError(RuntimeError):
    """The broker refused an operation (e.g. a publish over the maximum payload, no
    stream for a subject): a property of the request, not of the connection."""


class BusUnavailable(BusError, ConnectionError):
    """The broker could not be reached (connection closed / reset, no responders,
    timeout) or refuses EVERY request for now (stream full, resource limits, no
    leader, no stream for the subject).  Not any message's fault: the consume loop
    naks the batch whole (runtime/stage.py TRANSIENT) instead of isolating and
    dead-lettering."""


# Refusals that hit every message alike: JetStream's publish-ack errors
# for a full DiscardNew stream, resource limits, a leader election / cluster outage,
# and a subject no stream captures.  A refusal about ONE message (its payload over
# the maximum size, a malformed request) stays a plain BusError.
_BROKER_WIDE = re.compile(
    r"insufficient (storage |system )?resources|maximum (messages|bytes|consumers|streams)( per subject)? exceeded"
    r"|resource limits|no (stream|responders)|stream not found|not enabled|leader|cluster|temporarily unavailable"
    r"|unavailable|jetstream.*(offline|not ready)|503|no space left|storage full|stream (is )?full", re.I)


def bus_error(desc: str) -> BusError:
    """The exception for a broker's refusal ``desc``: :class:`BusUnavailable` when the
    condition is broker-wide (every message would fail alike), else :class:`BusError`."""
    return BusUnavailable(desc) if _BROKER_WIDE.search(desc or "") else BusError(desc)


class DeliverPolicy(str, enum.Enum):
    ALL = "all"
    NEW = "new"
    LAST = "last"


@dataclass
class StreamConfig:
    name: str
    subjects: List[str]
    max_age: float = 0.0  # seconds; 0 = unlimited
    max_msgs: int = -1
    max_bytes: int = -1
    storage: str = "file"  # "file" | "memory" (memory bus ignores it)


@dataclass
class ConsumerConfig:
    durable: str
    filter_subject: str = ">"
    ack_wait: float = 30.0
    max_deliver: int = -1
    deliver_policy: DeliverPolicy = DeliverPolicy.ALL
    max_ack_pending: int = 65536

    def __post_init__(self) -> None:
        self.deliver_policy = DeliverPolicy(self.deliver_policy)


@dataclass(slots=True)  # one per published message
class PubAck:
    stream: str
    seq: int
    duplicate: bool = False


@dataclass
class StreamInfo:
    config: StreamConfig
    messages: int
    bytes: int
    first_seq: int
    last_seq: int
    consumers: int


@dataclass
class ConsumerInfo:
    stream: str
    name: str
    num_pending: int  # stored, matching, never delivered
    num_ack_pending: int  # delivered, not yet acked
    num_redelivered: int
    delivered_seq: int
    ack_floor: int
    num_waiting: int = 0


def subject_matches(pattern: str, subject: str) -> bool:
    """NATS-style matching: ``*`` = one token, ``>`` = one or more trailing tokens."""
    if pattern == subject or pattern == ">":
        return True
    pt = pattern.split(".")
    st = subject.split(".")
    for i, tok in enumerate(pt):
        if tok == ">":
            return len(st) > i
        if i >= len(st):
            return False
        if tok != "*" and tok != st[i]:
            return False
    return len(pt) == len(st)


def default_stream_config(max_age: float = 3 * 24 * 3600.0) -> StreamConfig:
    """The reference's ``SMS`` stream (nats_utils.py:64-76): LIMITS, 3-day max_age."""
    return StreamConfig(name=STREAM_NAME, subjects=list(ALL_SUBJECTS), max_age=max_age)


@dataclass(slots=True)  # one per delivered message: no per-instance dict
class MsgMetadata:
    sequence: int
    num_delivered: int
    timestamp: float
    stream: str
    consumer: str


class Msg:
    """One delivered message.  ``data`` is bytes; ack/nak/term are idempotent.  The
    delivery metadata is kept as plain slots (one object per delivered message, not
    two); ``metadata`` builds the :class:`MsgMetadata` view when asked."""

    __slots__ = ("subject", "data", "headers", "_acker", "_done", "_seq", "_nd", "_ts", "_stream", "_consumer")

    def __init__(self, subject: str, data: bytes, metadata: MsgMetadata, acker: "Acker",
                 headers: Optional[Dict[str, str]] = None) -> None:
        self.subject = subject
        self.data = data
        self.headers = headers or {}
        self._acker = acker
        self._done = False
        self._seq, self._nd, self._ts = metadata.sequence, metadata.num_delivered, metadata.timestamp
        self._stream, self._consumer = metadata.stream, metadata.consumer

    @classmethod
    def delivered(cls, subject: str, data: bytes, seq: int, num_delivered: int, timestamp: float, stream: str,
                  consumer: str, acker: "Acker", headers: Optional[Dict[str, str]] = None) -> "Msg":
        """A message straight from a fetch reply's fields (no MsgMetadata built)."""
        m = cls.__new__(cls)
        m.subject, m.data, m.headers, m._acker, m._done = subject, data, headers or {}, acker, False
        m._seq, m._nd, m._ts, m._stream, m._consumer = seq, num_delivered, timestamp, stream, consumer
        return m

    @property
    def metadata(self) -> MsgMetadata:
        return MsgMetadata(self._seq, self._nd, self._ts, self._stream, self._consumer)

    @property
    def seq(self) -> int:
        return self._seq

    @property
    def settled(self) -> bool:
        """Already acked / nak'ed / terminated by this holder."""
        return self._done

    async def ack(self) -> None:
        if not self._done:
            self._done = True
            await self._acker.ack(self._stream, self._consumer, self._seq)

    async def nak(self, delay: float = 0.0) -> None:
        if not self._done:
            self._done = True
            await self._acker.nak(self._stream, self._consumer, self._seq, delay)

    async def term(self) -> None:
        if not self._done:
            self._done = True
            await self._acker.term(self._stream, self._consumer, self._seq)

    async def in_progress(self) -> None:
        if not self._done:
            await self._acker.touch(self._stream, self._consumer, self._seq)

    def json(self):
        import json

        return json.loads(self.data)

    def __repr__(self) -> str:  # pragma: no cover
        return f"Msg(subject={self.subject!r}, seq={self.seq}, len={len(self.data)})"


async def ack_all(msgs: Sequence["Msg"]) -> None:
    """Ack every unsettled message of a batch: one call per acker / consumer instead of
    one coroutine per message (an acker without ``ack_seqs`` gets them one by one)."""
    groups: Dict[Tuple[int, str, str], Tuple["Acker", List[int]]] = {}
    for m in msgs:
        if m._done:
            continue
        m._done = True
        key = (id(m._acker), m._stream, m._consumer)
        g = groups.get(key)
        if g is None:
            g = groups[key] = (m._acker, [])
        g[1].append(m._seq)
    for (_, stream, consumer), (acker, seqs) in groups.items():
        fn = getattr(acker, "ack_seqs", None)
        if fn is not None:
            await fn(stream, consumer, seqs)
        else:
            for q in seqs:
                await acker.ack(stream, consumer, q)


class Acker(abc.ABC):
    @abc.abstractmethod
    async def ack(self, stream: str, consumer: str, seq: int) -> None: ...

    @abc.abstractmethod
    async def nak(self, stream: str, consumer: str, seq: int, delay: float) -> None: ...

    @abc.abstractmethod
    async def term(self, stream: str, consumer: str, seq: int) -> None: ...

    @abc.abstractmethod
    async def touch(self, stream: str, consumer: str, seq: int) -> None: ...


class Subscription(abc.ABC):
    """A binding to a durable consumer.  Several may share one durable."""

    consumer: str

    @abc.abstractmethod
    async def fetch(self, batch: int = 1, timeout: Optional[float] = None) -> List[Msg]:
        """Wait up to ``timeout`` (None = forever) for >=1 message, return <= batch."""

    async def next_msg(self, timeout: Optional[float] = None) -> Optional[Msg]:
        got = await self.fetch(1, timeout)
        return got[0] if got else None

    @property
    def messages(self) -> AsyncIterator[Msg]:
        return self._iter()

    async def _iter(self) -> AsyncIterator[Msg]:
        while True:
            for m in await self.fetch(64, None):
                yield m

    @abc.abstractmethod
    async def unsubscribe(self) -> None: ...


class Bus(abc.ABC):
    """Durable subject bus (the NATS JetStream role)."""

    @abc.abstractmethod
    async def ensure_stream(self, config: Optional[StreamConfig] = None) -> StreamInfo: ...

    @abc.abstractmethod
    async def publish(self, subject: str, data: bytes, headers: Optional[Dict[str, str]] = None) -> PubAck: ...

    async def publish_many(self, items: Sequence[Tuple[str, bytes]]) -> List[PubAck]:
        return [await self.publish(s, d) for s, d in items]

    @abc.abstractmethod
    async def subscribe(self, subject: str, durable: str, **consumer_opts) -> Subscription: ...

    @abc.abstractmethod
    async def consumer_info(self, stream: str, durable: str) -> ConsumerInfo: ...

    @abc.abstractmethod
    async def stream_info(self, stream: str) -> StreamInfo: ...

    @abc.abstractmethod
    async def ping(self) -> bool: ...

    async def drain(self) -> None:
        await self.close()

    @abc.abstractmethod
    async def close(self) -> None: ...

    @property
    def is_connected(self) -> bool:
        return True


def now() -> float:
    return time.time()

