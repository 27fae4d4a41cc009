"""Prometheus metrics of every service, under the reference's metric names.

Parser worker (services/parser_worker/metrics.py:27-59) — served on
``PARSER_METRICS_PORT`` (default 9102; the reference read ``METRICS_PORT``
instead, metrics.py:109, and ``METRICS_PORT`` is still honoured):
``sms_parsed_ok_total``, ``sms_parsed_fail_total``, ``sms_parsed_skip_total``,
``sms_parser_stream_lag`` (now actually set from ``num_pending``),
``sms_parser_processing_seconds`` (1 ms…5 s buckets), ``sms_parser_gemini_seconds``
(the backend-call latency, whatever the backend), ``sms_parser_ack_pending``.

Writer (services/pb_writer/writer.py:35-39, port 9103):
``pb_writer_parsed_ok_total``, ``pb_writer_parsed_fail_total``, ``pb_writer_stream_lag``.

Gateway (new — README.md:37 promised port 9101 but nothing was exported, D12):
``api_gateway_requests_total{endpoint,status}``, ``api_gateway_publish_seconds``.

Local LLM engine (new; ``engine-server`` on ``ENGINE_METRICS_PORT``, default 9104,
exported by :class:`EngineMetricsExporter` from the engine's counters):
``llm_batch_size`` (decode rows per step), ``llm_step_seconds{phase}``,
``llm_tokens_total{phase}``, ``llm_sequences_completed_total``,
``llm_active_sequences``, ``llm_waiting_sequences``.
"""
from __future__ import annotations

import contextlib
import logging
import os
import threading
from typing import Optional

from prometheus_client import (
    REGISTRY,
    CollectorRegistry,
    Counter,
    Gauge,
    Histogram,
    Summary,
    generate_latest,
    start_http_server,
)

__all__ = [
    "PARSED_OK",
    "PARSED_FAIL",
    "PARSED_SKIP",
    "STREAM_LAG",
    "PROCESSING_TIME",
    "GEMINI_LATENCY",
    "observe_many",
    "ACK_PENDING",
    "WRITER_OK",
    "WRITER_FAIL",
    "WRITER_LAG",
    "GATEWAY_REQUESTS",
    "GATEWAY_PUBLISH_TIME",
    "LLM_BATCH",
    "LLM_STEP_TIME",
    "LLM_TOKENS",
    "LLM_COMPLETED",
    "LLM_ACTIVE",
    "LLM_WAITING",
    "LLM_TRUNCATED",
    "EngineMetricsExporter",
    "start_metrics_server",
    "render_latest",
]

log = logging.getLogger(__name__)

PARSED_OK = Counter("sms_parsed_ok_total", "SMS successfully parsed (or skipped as non-transaction)")
PARSED_FAIL = Counter("sms_parsed_fail_total", "SMS sent to the DLQ by the parser")
PARSED_SKIP = Counter("sms_parsed_skip_total", "SMS skipped as broken (no card)")
STREAM_LAG = Gauge("sms_parser_stream_lag", "Messages waiting for the parser consumer group")
PROCESSING_TIME = Histogram(
    "sms_parser_processing_seconds",
    "Seconds spent parsing one message",
    buckets=(0.001, 0.01, 0.05, 0.1, 0.25, 0.5, 1, 2, 5),
)
LLM_TRUNCATED = Counter("llm_prompt_truncated_total",
                        "SMS bodies cut to the extractor's max_body_tokens before extraction")
GEMINI_LATENCY = Summary("sms_parser_gemini_seconds", "Seconds spent in the extraction backend call")
ACK_PENDING = Gauge("sms_parser_ack_pending", "Delivered-but-unacked messages of the parser consumer")

DLQ_REPARSE_FAILED = Counter("sms_dlq_reparse_failed_total",
                             "DLQ messages whose reparse failed again (moved to sms.failed.final)")
WRITER_OK = Counter("pb_writer_parsed_ok_total", "Records saved by the writer")
WRITER_FAIL = Counter("pb_writer_parsed_fail_total", "Records the writer failed to save")
WRITER_LAG = Gauge("pb_writer_stream_lag", "sms.parsed consumer lag (messages)")

GATEWAY_REQUESTS = Counter("api_gateway_requests_total", "HTTP requests", ["endpoint", "status"])
GATEWAY_PUBLISH_TIME = Histogram("api_gateway_publish_seconds", "Seconds to publish one SMS to the bus")

LLM_BATCH = Histogram("llm_batch_size", "Sequences per extraction batch", buckets=(1, 8, 32, 64, 128, 256, 512, 1024, 2048))
LLM_STEP_TIME = Histogram("llm_step_seconds", "Seconds per engine step", ["phase"],
                          buckets=(1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 0.3, 1.0))
LLM_TOKENS = Counter("llm_tokens_total", "Tokens processed by the local extractor", ["phase"])
LLM_COMPLETED = Counter("llm_sequences_completed_total", "Extractions finished by the local engine")
LLM_ACTIVE = Gauge("llm_active_sequences", "Sequences decoding in the engine")
LLM_WAITING = Gauge("llm_waiting_sequences", "Sequences queued for prefill")


class EngineMetricsExporter:
    """Publishes an :class:`~smsgate_amd.serving.engine.ExtractionEngine`'s counters
    (``engine.stats``) as Prometheus metrics from a daemon thread, every
    ``interval`` seconds — the engine loop itself never touches prometheus_client."""

    def __init__(self, engine, interval: float = 1.0) -> None:
        self.engine = engine
        self.interval = interval
        self._last = dict(engine.stats.as_dict())
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="engine-metrics", daemon=True)

    def start(self) -> "EngineMetricsExporter":
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def export_once(self) -> None:
        cur = dict(self.engine.stats.as_dict())
        d = {k: v - self._last.get(k, 0) for k, v in cur.items()}
        d.setdefault("steps", 0)
        self._last = cur
        if d.get("prefill_tokens", 0) > 0:
            LLM_TOKENS.labels(phase="prefill").inc(d["prefill_tokens"])
        if d.get("decode_row_steps", 0) > 0:
            LLM_TOKENS.labels(phase="decode").inc(d["decode_row_steps"])
        if d.get("completed", 0) > 0:
            LLM_COMPLETED.inc(d["completed"])
        if d.get("decode_steps", 0) > 0:
            LLM_BATCH.observe(d["decode_row_steps"] / d["decode_steps"])
        if d["steps"] > 0:
            LLM_STEP_TIME.labels(phase="step").observe(d.get("step_s", 0.0) / d["steps"])
        LLM_ACTIVE.set(len(getattr(self.engine, "active", ()) or ()))
        LLM_WAITING.set(len(getattr(self.engine, "waiting", ()) or ()))

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self.export_once()
            except Exception:  # noqa: BLE001 — metrics must never take the engine down
                log.debug("engine metrics export failed", exc_info=True)

_started: set[int] = set()
_lock = threading.Lock()


def start_metrics_server(port: Optional[int] = None, *, env_var: str = "METRICS_PORT",
                         default: int = 9102, registry: CollectorRegistry = REGISTRY) -> Optional[int]:
    """Serve ``/metrics`` from a daemon thread; idempotent per port.

    Returns the port, or ``None`` if it could not be bound (the reference also
    swallowed ``OSError`` here, metrics.py:110).
    """
    if port is None:
        port = int(os.getenv(env_var, default))
    with _lock:
        if port in _started:
            return port
        with contextlib.suppress(OSError):
            start_http_server(port, registry=registry)
            _started.add(port)
            log.info("Prometheus metrics on :%s/metrics", port)
            return port
    return None


def render_latest(registry: CollectorRegistry = REGISTRY) -> bytes:
    """The exposition text.  Under ``PROMETHEUS_MULTIPROC_DIR`` (a multi-process
    server: ``gateway --workers N``) the counters of every worker process are
    aggregated, so ``/metrics`` is the same whichever worker answers it."""
    mp_dir = os.getenv("PROMETHEUS_MULTIPROC_DIR")
    if mp_dir and registry is REGISTRY:
        from prometheus_client import multiprocess

        reg = CollectorRegistry()
        multiprocess.MultiProcessCollector(reg, path=mp_dir)
        return generate_latest(reg)
    return generate_latest(registry)


def observe_many(metric, value: float, n: int) -> None:
    """``n`` observations of one ``value`` (the per-message latency of a batch, worker.py
    :130-133 observed once per message) in O(1): the same counters ``n`` observe() calls
    leave -- count / sum, and the one bucket the value falls in -- without n lock
    round trips.  Falls back to the loop for metric types it does not know."""
    if n <= 0:
        return
    try:
        if isinstance(metric, Histogram):
            import bisect

            i = bisect.bisect_left(metric._upper_bounds, value)
            metric._sum.inc(value * n)
            metric._buckets[i].inc(n)
            return
        if isinstance(metric, Summary):
            metric._count.inc(n)
            metric._sum.inc(value * n)
            return
    except AttributeError:
        pass
    for _ in range(n):
        metric.observe(value)
