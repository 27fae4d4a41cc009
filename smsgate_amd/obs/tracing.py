"""Lightweight transaction/span tracing.

The reference wraps each parsed message in a Sentry transaction
``task/process_parsing`` with spans ``check_stream``, ``validate``,
``parsing``, ``validate_parsed``, ``publish`` (worker.py:33-55, :80-171).
Here spans are recorded by an in-process :class:`Tracer` (per-span count and
total/max duration, cheap enough for the hot path) and forwarded to Sentry when
the SDK is active.  ``SMSGATE_TRACE=0`` disables recording entirely.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from dataclasses import dataclass
from typing import Dict, Iterator, Optional

from . import errors

__all__ = ["Tracer", "tracer", "start_transaction", "start_span", "SpanStats", "Profiler"]


@dataclass
class SpanStats:
    count: int = 0
    total_s: float = 0.0
    max_s: float = 0.0
    items: int = 0  # messages covered (a batch transaction covers many)

    @property
    def mean_s(self) -> float:
        return self.total_s / self.count if self.count else 0.0


class Tracer:
    def __init__(self, enabled: bool = True) -> None:
        self.enabled = enabled
        self._stats: Dict[str, SpanStats] = {}
        self._lock = threading.Lock()

    def record(self, name: str, dt: float, items: int = 1) -> None:
        with self._lock:
            s = self._stats.get(name)
            if s is None:
                s = self._stats[name] = SpanStats()
            s.count += 1
            s.items += items
            s.total_s += dt
            if dt > s.max_s:
                s.max_s = dt

    @contextlib.contextmanager
    def span(self, name: str, items: int = 1) -> Iterator[None]:
        if not self.enabled:
            yield
            return
        t0 = time.perf_counter()
        sdk = errors._sdk
        cm = sdk.start_span(name=name) if sdk is not None else contextlib.nullcontext()
        try:
            with cm:
                yield
        finally:
            self.record(name, time.perf_counter() - t0, items)

    def snapshot(self) -> Dict[str, SpanStats]:
        with self._lock:
            return {k: SpanStats(v.count, v.total_s, v.max_s, v.items) for k, v in self._stats.items()}

    def reset(self) -> None:
        with self._lock:
            self._stats.clear()


tracer = Tracer(enabled=os.getenv("SMSGATE_TRACE", "1") != "0")


@contextlib.contextmanager
def start_transaction(op: str, name: str, messages: Optional[int] = None) -> Iterator[None]:
    """One transaction; ``messages`` = how many SMS it covers.  The reference opens
    one per message (worker.py:33-55, :80); a batched handler opens one per batch
    and tags it with the message count (``sms.messages`` tag and data on the Sentry
    transaction, ``items`` in the local span stats), so per-message rates are
    recoverable from either side."""
    sdk = errors._sdk
    cm = sdk.start_transaction(op=op, name=name) if sdk is not None else contextlib.nullcontext()
    n = 1 if messages is None else int(messages)
    with cm as txn, tracer.span(f"{op}/{name}", items=n):
        if messages is not None and txn is not None:
            for setter, key in (("set_tag", "sms.messages"), ("set_data", "sms.messages")):
                fn = getattr(txn, setter, None)
                if fn is not None:
                    try:
                        fn(key, n)
                    except Exception:  # noqa: BLE001 — tracing must never break the handler
                        pass
        yield


def start_span(name: str, t: Optional[Tracer] = None):
    return (t or tracer).span(name)


class Profiler:
    """Host-side profiler session around a unit of work.

    The reference wraps DLQ reparse in ``sentry_sdk.profiler.start_profiler()``
    / ``stop_profiler()`` (dlq_worker.py:70-74).  Here the Sentry continuous
    profiler is started when the SDK is active; independently, when
    ``SMSGATE_PROFILE_DIR`` (or ``out_dir``) is set, a :mod:`cProfile` session
    runs and its stats are dumped to ``<dir>/<name>-<pid>.pstats`` on
    :meth:`stop` (readable with :mod:`pstats` or snakeviz).  With neither, the
    session costs nothing.  Re-entrant ``start`` calls are counted, so nested
    reparse batches share one session.
    """

    def __init__(self, name: str, out_dir: Optional[str] = None) -> None:
        self.name = name
        self.out_dir = out_dir if out_dir is not None else os.getenv("SMSGATE_PROFILE_DIR") or None
        self._depth = 0
        self._prof = None
        self._sentry = False
        self.dumped: Optional[str] = None

    def start(self) -> None:
        self._depth += 1
        if self._depth > 1:
            return
        sdk = errors._sdk
        prof_mod = getattr(sdk, "profiler", None) if sdk is not None else None
        if prof_mod is not None and hasattr(prof_mod, "start_profiler"):
            try:
                prof_mod.start_profiler()
                self._sentry = True
            except Exception:  # profiler not configured: keep going without it
                self._sentry = False
        if self.out_dir:
            import cProfile

            self._prof = cProfile.Profile()
            self._prof.enable()

    def stop(self) -> Optional[str]:
        if self._depth == 0:
            return None
        self._depth -= 1
        if self._depth > 0:
            return None
        if self._sentry:
            try:
                errors._sdk.profiler.stop_profiler()
            except Exception:
                pass
            self._sentry = False
        if self._prof is not None:
            self._prof.disable()
            os.makedirs(self.out_dir, exist_ok=True)
            path = os.path.join(self.out_dir, f"{self.name}-{os.getpid()}.pstats")
            self._prof.dump_stats(path)
            self._prof = None
            self.dumped = path
        return self.dumped

    def __enter__(self) -> "Profiler":
        self.start()
        return self

    def __exit__(self, *exc) -> None:
        self.stop()
