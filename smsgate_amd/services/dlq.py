"""DLQ inspector / re-parser (services/parser_worker/dlq_worker.py parity).

Consumes ``sms.failed`` as durable ``parser_worker_dlq`` (dlq_worker.py:84-90),
logs every envelope pretty-printed and, with ``--reparse``, runs the message
through the parse pipeline again.  Successes are routed like the parser worker
(``sms.parsed`` + ``sms.processing``); a message that fails again is logged,
counted (``reparse_failed``, Prometheus ``sms_dlq_reparse_failed_total``) and
moved to the terminal subject ``sms.failed.final`` (no consumer: kept for
inspection), never republished to ``sms.failed`` — this worker reads that
subject, so a republish would loop forever.

Fixes: every message is acked (the reference never acked
non-``raw`` payloads in reparse mode), and every envelope shape that carries
a RawSMS can be re-parsed — ``{"raw": RawSMS}`` (c), ``{"entry": RawSMS}``
(b) and ``{"entry": "<RawSMS JSON>"}`` (a, d, e) — not only shape (c).
Writer failures (f: ``entry`` is a ParsedSMS) are logged, not re-parsed.
"""
from __future__ import annotations

import json
import logging
from typing import Any, Dict, List, Optional, Sequence

from ..bus.base import SUBJECT_FAILED, SUBJECT_FAILED_FINAL, Bus, BusError, BusUnavailable, Msg
from ..obs.metrics import DLQ_REPARSE_FAILED
from ..models.domain import RawSMS
from ..obs.tracing import Profiler
from ..parse.pipeline import ParsePipeline
from ..runtime.stage import Stage, dlq_publisher

__all__ = ["DlqWorker", "extract_raw"]

log = logging.getLogger("dlq_worker")


def extract_raw(envelope: Any) -> Optional[Dict[str, Any]]:
    """The RawSMS dict inside a DLQ envelope, or None."""
    if not isinstance(envelope, dict):
        return None
    cand = envelope.get("raw", envelope.get("entry"))
    if isinstance(cand, str):
        try:
            cand = json.loads(cand)
        except ValueError:
            return None
    if isinstance(cand, dict) and "raw" in cand and isinstance(cand["raw"], dict):
        cand = cand["raw"]
    if not isinstance(cand, dict):
        return None
    try:
        RawSMS(**cand)
    except Exception:  # noqa: BLE001 — e.g. a writer-failure ParsedSMS entry
        return None
    return cand


class DlqWorker:
    def __init__(self, bus: Bus, pipeline: Optional[ParsePipeline] = None, *, group: str = "parser_worker_dlq",
                 reparse: bool = False, batch: int = 64) -> None:
        self.bus = bus
        self.pipeline = pipeline
        self.reparse = reparse
        self.seen = 0
        self.reparsed = 0
        self.not_reparsable = 0
        self.reparse_failed = 0
        self.final_rejected = 0  # twice-failed messages the broker refused on the terminal subject
        self.log: List[Dict[str, Any]] = []
        # reparse runs under a profiler session (dlq_worker.py:70-74)
        self.profiler = Profiler("dlq_reparse")
        # a message whose handling keeps failing (not a transient outage: those nak) ends
        # on the terminal subject after poison_after deliveries, never silently dropped
        self.stage = Stage(bus, SUBJECT_FAILED, group, self.handle_batch, batch=batch, stats_interval=0,
                           name="dlq_worker", dead_letter=dlq_publisher(bus, SUBJECT_FAILED_FINAL))

    async def handle_batch(self, msgs: Sequence[Msg]) -> None:
        from ..services.parser import route_batch

        to_reparse: List[Msg] = []
        for m in msgs:
            self.seen += 1
            try:
                env = json.loads(m.data)
            except ValueError:
                log.error("DLQ payload is not JSON: %r", m.data[:120])
                continue
            log.info("DLQ seq=%s payload=%s", m.seq, json.dumps(env, ensure_ascii=False, indent=2))
            self.log.append(env)
            if self.reparse:
                raw = extract_raw(env)
                if raw is None:
                    self.not_reparsable += 1
                else:
                    to_reparse.append(_Shim(json.dumps({"raw": raw}).encode()))
        if to_reparse and self.pipeline is not None:
            with self.profiler:
                publishes, counts = await route_batch(self.pipeline, to_reparse)
                # Only successes leave the DLQ.  A message that fails again is
                # logged and acked here, never republished to sms.failed: this
                # worker consumes that subject, so a republish would re-feed it
                # forever (and re-call the backend on every lap).
                keep = [(s, p) for s, p in publishes if s != SUBJECT_FAILED]
                final = []
                for s, p in publishes:
                    if s == SUBJECT_FAILED:
                        self.reparse_failed += 1
                        DLQ_REPARSE_FAILED.inc()
                        log.warning("DLQ reparse failed again (moved to %s): %s", SUBJECT_FAILED_FINAL, p[:300])
                        final.append((SUBJECT_FAILED_FINAL, p))
                if keep:
                    await self.bus.publish_many(keep)
                if final:
                    try:
                        await self.bus.publish_many(final)
                    except BusUnavailable:
                        raise  # broker gone: the stage naks the batch and retries it
                    except BusError as exc:
                        # the broker refuses the terminal subject (e.g. a reference-created
                        # stream whose subject list could not be updated): log and ack --
                        # retrying cannot succeed and must not pin the DLQ consumer
                        self.final_rejected += len(final)
                        log.error("DLQ: %s rejected %d twice-failed message(s), logged and acked: %s",
                                  SUBJECT_FAILED_FINAL, len(final), exc)
                        for _, p in final:
                            log.error("DLQ twice-failed payload: %s", p[:2000])
            self.reparsed += len(to_reparse)
        for m in msgs:
            await m.ack()

    async def start(self) -> None:
        await self.bus.ensure_stream()
        await self.stage.start()

    async def stop(self) -> None:
        await self.stage.stop()


class _Shim:
    """Minimal Msg stand-in for re-routing an extracted RawSMS."""

    def __init__(self, data: bytes) -> None:
        self.data = data
