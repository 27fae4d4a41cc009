"""Writer service: ``sms.parsed`` → sinks (PocketBase + SQL), ``pb_writer`` parity.

Per message (writer.py:65-84): validate as :class:`ParsedSMS`; only records
with a truthy ``merchant`` are stored (:70 — kept: skipped records are acked
and counted nowhere, as in the reference); a future date fails with
``"Bad date"``; storage is retried 5× with exponential backoff 1–20 s
(:57-62); any failure → ``pb_writer_parsed_fail_total``, error capture and a
``{"err", "entry": <payload>}`` envelope on ``sms.failed`` (shape f); every
message is acked.

Batched: a batch is written with one upsert per sink; if that fails after its
retries, records are retried one by one so a single poison record only fails
itself.  Sinks are written in order (PocketBase first, then SQL, like
writer.py:60-61) and SQL errors are *not* swallowed (D4).
"""
from __future__ import annotations

import asyncio
import json
import logging
from datetime import datetime, timezone
from typing import List, Optional, Sequence, Tuple

from ..bus.base import SUBJECT_FAILED, SUBJECT_PARSED, Bus, Msg, ack_all
from ..models.domain import LazyParsedSMS, ParsedSMS
from ..parse import fastpath
from ..obs import metrics as M
from ..obs.errors import sentry_capture
from ..runtime.retry import retry
from ..runtime.stage import Stage, dlq_publisher
from ..sinks.base import Sink

__all__ = ["WriterService"]

log = logging.getLogger("pb_writer")


def _future(dt: datetime) -> bool:
    return dt > (datetime.now(timezone.utc) if dt.tzinfo else datetime.now())


class WriterService:
    def __init__(self, bus: Bus, sinks: Sequence[Sink], *, durable: str = "pb_writer", batch: int = 128,
                 retry_attempts: int = 5, retry_min: float = 1.0, retry_max: float = 20.0,
                 stats_interval: float = 1.0, ack_wait: float = 30.0) -> None:
        self.bus = bus
        self.sinks = list(sinks)
        self.ok = 0
        self.fail = 0
        self.skipped = 0
        self._upsert = retry(attempts=retry_attempts, wait_min=retry_min, wait_max=retry_max)(self._upsert_all)
        self.stage = Stage(bus, SUBJECT_PARSED, durable, self.handle_batch, batch=batch,
                           stats_interval=stats_interval, ack_wait=ack_wait, on_stats=lambda p, a: M.WRITER_LAG.set(p),
                           name="pb_writer", dead_letter=dlq_publisher(bus, SUBJECT_FAILED))

    async def _upsert_all(self, records: Sequence[ParsedSMS]) -> None:
        for s in self.sinks:
            await s.upsert_many(records)

    async def handle_batch(self, msgs: Sequence[Msg]) -> None:
        dlq: List[Tuple[str, bytes]] = []
        to_store: List[Tuple[ParsedSMS, str]] = []

        def fail(err: BaseException, text: str) -> None:
            self.fail += 1
            M.WRITER_FAIL.inc()
            sentry_capture(err, extras={"raw_msg": text})
            dlq.append((SUBJECT_FAILED, json.dumps({"err": str(err), "entry": text}).encode()))

        datas = [m.data for m in msgs]
        # the canonical payloads (what the parser writes) are checked natively and stored
        # as LazyParsedSMS records: no second pydantic pass over bytes just produced
        peek = fastpath.peek_parsed([d if isinstance(d, bytes) else b"" for d in datas])
        now = None
        for data, pk in zip(datas, peek):
            if pk is not None:
                msg_id, has_merchant, dt = pk
                if not has_merchant:
                    self.skipped += 1
                    continue
                if now is None:
                    n = datetime.now()
                    now = (n.year, n.month, n.day, n.hour, n.minute, n.second, n.microsecond)
                if dt > now[:6]:  # naive date in the future (equal seconds: not after now)
                    fail(ValueError("Bad date"), data.decode(errors="ignore"))
                    continue
                to_store.append((LazyParsedSMS(msg_id, data), data))
                continue
            try:
                # one Rust pass parses and validates the bytes (the reference: json +
                # model_validate); the text is decoded only for a failure envelope
                p = ParsedSMS.model_validate_json(data)
                if not p.merchant:
                    self.skipped += 1
                    continue
                if _future(p.date):
                    raise ValueError("Bad date")
                to_store.append((p, data))
            except Exception as err:  # noqa: BLE001
                fail(err, data.decode(errors="ignore") if isinstance(data, (bytes, bytearray)) else str(data))

        if to_store:
            try:
                await self._upsert([p for p, _ in to_store])
                stored = len(to_store)
            except Exception:
                stored = 0
                for p, text in to_store:
                    try:
                        await self._upsert([p])
                        stored += 1
                    except Exception as err:  # noqa: BLE001
                        fail(err.__cause__ or err, text.decode(errors="ignore")
                             if isinstance(text, (bytes, bytearray)) else str(text))
            self.ok += stored
            if stored:
                M.WRITER_OK.inc(stored)

        if dlq:
            await self.bus.publish_many(dlq)
        await ack_all(msgs)

    async def start(self) -> None:
        await self.bus.ensure_stream()
        for s in self.sinks:
            await s.start()
        await self.stage.start()

    async def stop(self) -> None:
        await self.stage.stop()
        for s in self.sinks:
            await s.close()

    async def run(self, stop: Optional[asyncio.Event] = None) -> None:
        await self.start()
        try:
            await (stop.wait() if stop is not None else asyncio.Event().wait())
        finally:
            await self.stop()
