"""The consume → handle → ack runtime shared by every worker service.

The reference copy-pastes one serial loop per service
(``async for msg in sub.messages: await _process_one(...)`` — worker.py:206,
writer.py:108, dlq_worker.py:89) and an exception escaping ``_process_one``
silently kills that loop while the process stays up (D1/D2).  :class:`Stage`
is the one loop, written once:

* pulls *batches* from a durable competing consumer (``batch`` ≤ backend max);
* runs up to ``concurrency`` batch handlers at once (I/O-bound handlers such as
  a remote LLM or a database get overlap; a GPU handler gets a full batch);
* never dies on a handler exception (D1/D2), and bounds poison messages:

  - a :class:`~smsgate_amd.runtime.errors.TransientError` (engine restarting,
    socket closed, its request timed out), a ``BusUnavailable`` /
    ``ConnectionError`` (the broker went away mid-batch, timed out, or refuses every
    request for now: stream full, resource limits, no leader, no stream for the
    subject -- ``bus.base.bus_error``) naks the whole batch with a delay — not the
    messages' fault, so it never counts toward dead-lettering.  A plain
    ``BusError`` is the broker refusing ONE request (a publish over the maximum
    payload): that is a property of a message and takes the isolate / dead-letter
    path below, so it cannot pin its batch forever; so does any other timeout;
  - any other exception re-runs the batch one message at a time, so the good
    messages of the batch go through and only the failing one is isolated;
    that one is nak'ed with a delay until it has been delivered
    ``poison_after`` times, then handed to ``dead_letter`` (the parser
    publishes a DLQ envelope) and terminated — it never redelivers forever
    (the reference acked every handled branch, worker.py:109-189, but an
    *unhandled* exception killed its loop);
* exports lag/ack-pending gauges from ``consumer_info`` on a timer;
* drains in-flight batches on stop (graceful shutdown, worker.py:241-263).
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Awaitable, Callable, List, Optional, Sequence

from ..bus.base import Bus, BusUnavailable, Msg, Subscription
from ..obs.errors import sentry_capture
from .errors import TransientError

__all__ = ["Stage", "BatchHandler", "dlq_publisher", "TRANSIENT"]

log = logging.getLogger(__name__)

# not the messages' fault: the batch is nak'ed whole (never split into per-message
# re-runs, never counted toward dead-lettering) -- a dependency (engine, broker) is
# down, refuses every request for now (stream full, no leader: bus.base.bus_error), or
# the connection broke mid-batch.  (BusUnavailable is a ConnectionError; a plain
# BusError -- the broker refused ONE request -- is not here.)  Timeouts are not here
# either: the bus and engine clients turn THEIR timeouts into
# BusUnavailable / BackendUnavailable; any other TimeoutError (a handler timing out the
# same way on one message every time) takes the isolate / dead-letter path, so it
# cannot pin its batch forever.
TRANSIENT = (TransientError, BusUnavailable, ConnectionError)

# a dead-letter envelope carries at most this much of the failed payload: the payload
# may be what the broker refused (over its maximum size), and the envelope must fit
DLQ_ENTRY_MAX = 64 * 1024

BatchHandler = Callable[[Sequence[Msg]], Awaitable[None]]
DeadLetter = Callable[[Msg, BaseException], Awaitable[None]]


def dlq_publisher(bus: Bus, subject: str) -> DeadLetter:
    """Dead-letter callback publishing the ``{"err", "entry": <payload text>}``
    envelope (the reference's shapes a/d/f, worker.py:105, writer.py:80-82)."""
    import json

    async def publish(m: Msg, exc: BaseException) -> None:
        data = m.data if isinstance(m.data, (bytes, bytearray)) else str(m.data).encode()
        env = {"err": str(exc)[:4096], "entry": data[:DLQ_ENTRY_MAX].decode(errors="ignore")}
        if len(data) > DLQ_ENTRY_MAX:
            env["entry_truncated"] = len(data)  # original size; the entry holds its first DLQ_ENTRY_MAX bytes
        await bus.publish(subject, json.dumps(env).encode())

    return publish


class Stage:
    def __init__(
        self,
        bus: Bus,
        subject: str,
        durable: str,
        handler: BatchHandler,
        *,
        batch: int = 64,
        concurrency: int = 1,
        fetch_timeout: float = 0.5,
        ack_wait: float = 30.0,
        max_deliver: int = -1,
        nak_delay: float = 1.0,
        stats_interval: float = 5.0,
        on_stats: Optional[Callable[[int, int], None]] = None,
        name: Optional[str] = None,
        poison_after: int = 5,
        dead_letter: Optional[DeadLetter] = None,
        max_ack_pending: Optional[int] = None,
    ) -> None:
        self.bus = bus
        self.subject = subject
        self.durable = durable
        self.handler = handler
        self.batch = max(1, batch)
        self.concurrency = max(1, concurrency)
        self.fetch_timeout = fetch_timeout
        self.ack_wait = ack_wait
        self.max_deliver = max_deliver
        self.nak_delay = nak_delay
        self.stats_interval = stats_interval
        self.on_stats = on_stats
        self.name = name or durable
        self.max_ack_pending = max_ack_pending
        self.poison_after = poison_after
        self.dead_letter = dead_letter
        self.dead_lettered = 0
        self.transient_errors = 0
        self.sub: Optional[Subscription] = None
        self.processed = 0
        self.batches = 0
        self.handler_errors = 0
        self._stop = asyncio.Event()
        self._tasks: List[asyncio.Task] = []

    async def open(self) -> Subscription:
        if self.sub is None:
            opts = {"ack_wait": self.ack_wait, "max_deliver": self.max_deliver}
            if self.max_ack_pending is not None:
                opts["max_ack_pending"] = self.max_ack_pending
            self.sub = await self.bus.subscribe(self.subject, self.durable, **opts)
        return self.sub

    async def _worker(self, wid: int) -> None:
        sub = await self.open()
        while not self._stop.is_set():
            try:
                msgs = await sub.fetch(self.batch, self.fetch_timeout)
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # bus hiccup: back off, keep running
                log.warning("%s: fetch failed: %s", self.name, exc)
                sentry_capture(exc, extras={"stage": self.name})
                await asyncio.sleep(0.5)
                continue
            if not msgs:
                continue
            await self._run_batch(msgs)

    async def _run_batch(self, msgs: Sequence[Msg]) -> None:
        try:
            await self.handler(msgs)
        except asyncio.CancelledError:
            raise
        except TRANSIENT as exc:
            self.transient_errors += 1
            log.warning("%s: dependency unavailable, batch of %d nak'ed: %s", self.name, len(msgs), exc)
            await self._nak(msgs)
        except Exception as exc:
            self.handler_errors += 1
            log.exception("%s: handler failed on a batch of %d", self.name, len(msgs))
            sentry_capture(exc, extras={"stage": self.name, "batch": len(msgs)})
            if len(msgs) == 1:
                await self._failed(msgs[0], exc)
            else:
                await self._isolate(msgs)
        self.processed += len(msgs)
        self.batches += 1

    async def _nak(self, msgs: Sequence[Msg]) -> None:
        for m in msgs:
            try:
                await m.nak(self.nak_delay)
            except Exception:  # pragma: no cover — the bus redelivers after ack_wait anyway
                pass

    async def _isolate(self, msgs: Sequence[Msg]) -> None:
        """Re-run a failed batch one message at a time (skipping any the handler
        already settled before it raised)."""
        for i, m in enumerate(msgs):
            if m.settled:
                continue
            try:
                await self.handler([m])
            except asyncio.CancelledError:
                raise
            except TRANSIENT:
                self.transient_errors += 1
                await self._nak(msgs[i:])
                return
            except Exception as exc:  # noqa: BLE001
                await self._failed(m, exc)

    async def _failed(self, m: Msg, exc: BaseException) -> None:
        delivered = getattr(getattr(m, "metadata", None), "num_delivered", 1) or 1
        if self.poison_after <= 0 or delivered < self.poison_after:
            await self._nak([m])
            return
        self.dead_lettered += 1
        log.error("%s: message seq=%s failed %d deliveries, dead-lettered: %s", self.name,
                  getattr(m, "seq", "?"), delivered, exc)
        if self.dead_letter is not None:
            try:
                await self.dead_letter(m, exc)
            except Exception as dl_exc:  # noqa: BLE001 — keep it for a later delivery
                sentry_capture(dl_exc, extras={"stage": self.name})
                await self._nak([m])
                return
        try:
            await m.term()
        except Exception:  # pragma: no cover
            pass

    async def _stats(self) -> None:
        while not self._stop.is_set():
            try:
                stream = getattr(self.sub, "stream", None) or "SMS"
                info = await self.bus.consumer_info(stream, self.durable)
                if self.on_stats is not None:
                    self.on_stats(info.num_pending, info.num_ack_pending)
            except Exception as exc:  # noqa: BLE001
                log.debug("%s: stats failed: %s", self.name, exc)
            try:
                await asyncio.wait_for(self._stop.wait(), self.stats_interval)
            except asyncio.TimeoutError:
                pass

    async def start(self) -> None:
        await self.open()
        self._stop.clear()
        self._tasks = [asyncio.create_task(self._worker(i), name=f"{self.name}-w{i}")
                       for i in range(self.concurrency)]
        if self.on_stats is not None and self.stats_interval > 0:
            self._tasks.append(asyncio.create_task(self._stats(), name=f"{self.name}-stats"))

    async def stop(self, timeout: float = 10.0) -> None:
        """Stop fetching, let in-flight batches finish (bounded), then cancel."""
        self._stop.set()
        if not self._tasks:
            return
        done, pending = await asyncio.wait(self._tasks, timeout=timeout)
        for t in pending:
            t.cancel()
        for t in pending:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self._tasks = []

    async def run(self, stop: Optional[asyncio.Event] = None) -> None:
        await self.start()
        try:
            if stop is None:
                await asyncio.gather(*self._tasks)
            else:
                await stop.wait()
        finally:
            await self.stop()

    async def run_until_idle(self, idle_s: float = 0.2, max_s: float = 60.0) -> int:
        """Test/benchmark helper: process until no message arrives for ``idle_s``."""
        sub = await self.open()
        t_end = time.monotonic() + max_s
        n0 = self.processed
        while time.monotonic() < t_end:
            msgs = await sub.fetch(self.batch, idle_s)
            if not msgs:
                break
            await self._run_batch(msgs)
        return self.processed - n0
