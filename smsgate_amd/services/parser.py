"""Parser worker: ``sms.raw`` → parse → ``sms.parsed`` + ``sms.processing`` | ``sms.failed``.

Routing is exactly the reference's ``_process_one`` (worker.py:74-189;
SURVEY.md §3.2, envelope shapes §2.12), per message:

====================================  ==============================================  =========
condition                             published                                       metric
====================================  ==============================================  =========
payload not JSON / not a RawSMS       ``{"err", "entry": <payload str>}`` (a)         FAIL
worker keyword skip (OTP, C2C …)      nothing                                         OK (D11)
card missing (BrokenMessage)          nothing                                         SKIP
backend raised                        ``{"err", "entry": RawSMS dict}`` (b)           FAIL
unmatched / post-processing failed    ``{"reason": "unmatched", "raw": RawSMS}`` (c)  FAIL
ParsedSMS re-validation failed        ``{"err", "entry": <payload str>}`` (d)         FAIL
date in the future                    ``{"err": "Дата больше чем сегодня", …}`` (e)   FAIL
parsed                                ParsedSMS JSON on parsed *and* processing      OK
====================================  ==============================================  =========

Every branch acks (after its publish), so poison messages never loop.
A DLQ envelope carrying ``raw`` is unwrapped, so ``sms.failed`` entries can be
re-fed (dlq ``--reparse``).

Fixed defects: D1 (a malformed payload or future date no longer kills the
loop: the decoded text is kept separately from the bytes), D2 (tz-aware dates
are compared with an aware "now"), R4 (the backend is awaited — blocking
backends run in threads, GPU backends batch), D3 (the stream is ensured once
at start, not per message).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from datetime import datetime, timezone
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ..bus.base import SUBJECT_FAILED, SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_RAW, Bus, Msg, ack_all
from ..models.domain import RawSMS, parsed_wire
from ..obs import metrics as M
from ..obs.errors import sentry_capture
from ..obs.tracing import start_span, start_transaction
from ..parse import fastpath
from ..parse.pipeline import Outcome, ParsePipeline
from ..parse.text import worker_should_skip
from ..runtime.stage import Stage, dlq_publisher

__all__ = ["ParserWorker", "FUTURE_DATE_ERR", "route_batch"]

log = logging.getLogger("parser_worker")

FUTURE_DATE_ERR = "Дата больше чем сегодня"


def _is_future(dt: datetime) -> bool:
    if dt.tzinfo is None:
        return dt > datetime.now()
    return dt > datetime.now(timezone.utc)


def _text(data: bytes) -> str:
    return data.decode(errors="ignore")


def _dump(obj: Dict[str, Any]) -> bytes:
    return json.dumps(obj).encode()


async def route_batch(pipeline: ParsePipeline, msgs: Sequence[Msg]) -> Tuple[List[Tuple[str, bytes]], Dict[str, int]]:
    """Decide every message's output. Returns ``(publishes, counters)``."""
    out: List[Tuple[str, bytes]] = []
    # ok / fail / skip are the reference's metric semantics (a keyword skip counts as
    # ok, D11); parsed and keyword_skipped split "ok" into what actually happened
    counts = {"ok": 0, "fail": 0, "skip": 0, "parsed": 0, "keyword_skipped": 0}
    texts: List[bytes] = []
    raws: List[RawSMS] = []
    raw_idx: List[int] = []

    with start_span("validate"):
        datas = [m.data if isinstance(m.data, (bytes, bytearray)) else str(m.data).encode() for m in msgs]
        # the native scan (parse/fastpath.py): a valid RawSMS no keyword filter can touch,
        # body normalised -- or None, and the Python path below decides
        fast = fastpath.scan(datas)
        for i, data in enumerate(datas):
            texts.append(data)  # decoded only for a failure envelope (_text)
            if fast[i] is not None:
                raws.append(fast[i])
                raw_idx.append(i)
                continue
            try:
                if b'"raw"' not in data:
                    # fast path: pydantic-core parses + validates the JSON bytes in one
                    # pass (falls back below on any error, so failure routing is unchanged)
                    try:
                        raw = RawSMS.model_validate_json(data)
                    except Exception:
                        raw = None
                else:
                    raw = None
                if raw is None:
                    text = _text(data)
                    payload = json.loads(text)
                    if isinstance(payload, dict) and "raw" in payload:
                        payload = payload["raw"]
                    raw = RawSMS(**payload)
            except Exception as err:
                text = _text(data)
                out.append((SUBJECT_FAILED, _dump({"err": str(err), "entry": text})))
                counts["fail"] += 1
                sentry_capture(err, extras={"raw_data": text})
                continue
            if worker_should_skip(raw.body):
                counts["ok"] += 1
                counts["keyword_skipped"] += 1
                continue
            raws.append(raw)
            raw_idx.append(i)

    if raws:
        t0 = time.perf_counter()
        with start_span("parsing"):
            results = await pipeline.parse_batch(raws)
        # one observation per message (worker.py:131-133 times each message), so the
        # histogram's _count equals messages parsed; the value is the latency the
        # message experienced (the batched parse it was part of)
        M.observe_many(M.PROCESSING_TIME, time.perf_counter() - t0, len(raws))

        with start_span("validate_parsed"):
            for raw, i, res in zip(raws, raw_idx, results):
                data = texts[i]
                if res.outcome is Outcome.BROKEN:
                    counts["skip"] += 1
                    continue
                if res.outcome is Outcome.ERROR:
                    out.append((SUBJECT_FAILED, _dump({"err": str(res.error), "entry": raw.model_dump()})))
                    counts["fail"] += 1
                    continue
                if res.outcome is Outcome.UNMATCHED or (res.parsed is None and res.wire is None):
                    out.append((SUBJECT_FAILED, _dump({"reason": "unmatched", "raw": raw.model_dump()})))
                    counts["fail"] += 1
                    continue
                # The reference re-validated here (ParsedSMS(**parsed.model_dump()),
                # worker.py:161-170) — a no-op for an already-validated model, so
                # only the serialisation keeps the shape-(d) failure route.
                if res.wire is not None:  # the native path's payload (future dates excluded there)
                    out.append((SUBJECT_PARSED, res.wire))
                    out.append((SUBJECT_PROCESSING, res.wire))
                    counts["ok"] += 1
                    counts["parsed"] += 1
                    continue
                parsed = res.parsed
                try:
                    future = _is_future(parsed.date)
                except (ValueError, OverflowError) as err:  # an unusable date: this message's failure
                    text = _text(data)
                    sentry_capture(err, extras={"raw_data": text})
                    out.append((SUBJECT_FAILED, _dump({"err": str(err), "entry": text})))
                    counts["fail"] += 1
                    continue
                if future:
                    text = _text(data)
                    sentry_capture(ValueError(FUTURE_DATE_ERR), extras={"raw_data": text})
                    out.append((SUBJECT_FAILED, _dump({"err": FUTURE_DATE_ERR, "entry": text})))
                    counts["fail"] += 1
                    continue
                try:
                    payload = parsed_wire(parsed)
                except Exception as err:
                    text = _text(data)
                    sentry_capture(err, extras={"raw_data": text})
                    out.append((SUBJECT_FAILED, _dump({"err": str(err), "entry": text})))
                    counts["fail"] += 1
                    continue
                out.append((SUBJECT_PARSED, payload))
                out.append((SUBJECT_PROCESSING, payload))
                counts["ok"] += 1
                counts["parsed"] += 1
    return out, counts


class ParserWorker:
    """The parser service: one :class:`Stage` over ``sms.raw`` + a :class:`ParsePipeline`."""

    def __init__(self, bus: Bus, pipeline: ParsePipeline, *, group: str = "parser_worker",
                 batch: Optional[int] = None, concurrency: int = 1, ack_wait: float = 30.0,
                 stats_interval: float = 5.0) -> None:
        self.bus = bus
        self.pipeline = pipeline
        self.group = group
        self.counts = {"ok": 0, "fail": 0, "skip": 0, "parsed": 0, "keyword_skipped": 0}
        self.stage = Stage(
            bus,
            SUBJECT_RAW,
            group,
            self.handle_batch,
            batch=batch or pipeline.backend.max_batch,
            concurrency=concurrency,
            ack_wait=ack_wait,
            stats_interval=stats_interval,
            on_stats=self._on_stats,
            name="parser_worker",
            dead_letter=dlq_publisher(bus, SUBJECT_FAILED),
        )

    @staticmethod
    def _on_stats(num_pending: int, num_ack_pending: int) -> None:
        M.STREAM_LAG.set(num_pending)
        M.ACK_PENDING.set(num_ack_pending)

    async def handle_batch(self, msgs: Sequence[Msg]) -> None:
        with start_transaction("task", "process_parsing", messages=len(msgs)):
            publishes, counts = await route_batch(self.pipeline, msgs)
            with start_span("publish"):
                if publishes:
                    await self.bus.publish_many(publishes)
                await ack_all(msgs)
        if counts["ok"]:
            M.PARSED_OK.inc(counts["ok"])
        if counts["fail"]:
            M.PARSED_FAIL.inc(counts["fail"])
        if counts["skip"]:
            M.PARSED_SKIP.inc(counts["skip"])
        for k, v in counts.items():
            self.counts[k] += v

    async def start(self) -> None:
        await self.bus.ensure_stream()
        await self.pipeline.backend.start()
        await self.stage.start()

    async def stop(self) -> None:
        await self.stage.stop()
        await self.pipeline.backend.close()

    async def run(self, stop: Optional[asyncio.Event] = None) -> None:
        await self.start()
        try:
            await (stop.wait() if stop is not None else asyncio.Event().wait())
        finally:
            await self.stop()
