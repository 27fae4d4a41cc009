"""Sentry-compatible error capture (``libs/sentry.py:41-87`` of the reference).

* :func:`init_sentry` — once per process; a no-op unless ``ENABLE_SENTRY`` and
  a DSN are set *and* ``sentry_sdk`` is importable (it is not on the MI355X
  image). Sample rates come from ``SENTRY_TRACES_SAMPLE_RATE`` /
  ``SENTRY_PROFILE_SAMPLE_RATE`` (default 1.0), ``max_value_length=4096``.
* :func:`sentry_capture` — records the exception with ``extras``.

Unlike the reference, captures are never silently lost when the SDK is absent:
every capture also lands in an in-process ring buffer (inspectable by tests
and the ``/debug/errors`` endpoint) and, when ``SMSGATE_ERROR_LOG`` names a
file, as one JSON line per event — the offline fallback the legacy
``process_cached.py:68-83`` implemented with a diskcache.
"""
from __future__ import annotations

import collections
import json
import logging
import os
import threading
import time
import traceback
from typing import Any, Deque, Dict, List, Optional

__all__ = ["init_sentry", "sentry_capture", "recent_errors", "clear_errors", "sentry_enabled"]

log = logging.getLogger(__name__)

_lock = threading.Lock()
_ring: Deque[Dict[str, Any]] = collections.deque(maxlen=1024)
_initialised = False
_sdk = None  # the sentry_sdk module once initialised


def sentry_enabled() -> bool:
    return _sdk is not None


def init_sentry(*, release: Optional[str] = None, env: Optional[str] = None) -> bool:
    """Initialise the real SDK if possible; returns whether it is active."""
    global _initialised, _sdk
    with _lock:
        if _initialised:
            return _sdk is not None
        _initialised = True
        from ..config import get_settings

        settings = get_settings()
        if not settings.enable_sentry:
            return False
        dsn = os.getenv("SENTRY_DSN") or settings.sentry_dsn
        if not dsn:
            return False
        try:
            import sentry_sdk  # type: ignore
        except ImportError:
            log.warning("ENABLE_SENTRY is set but sentry_sdk is not installed; using the local error log")
            return False
        sentry_sdk.init(
            dsn=dsn,
            release=release,
            environment=env or "local",
            traces_sample_rate=float(os.getenv("SENTRY_TRACES_SAMPLE_RATE", "1.0")),
            profile_session_sample_rate=float(os.getenv("SENTRY_PROFILE_SAMPLE_RATE", "1.0")),
            max_value_length=4096,
        )
        _sdk = sentry_sdk
        return True


def _truncate(v: Any, limit: int = 4096) -> Any:
    if isinstance(v, str) and len(v) > limit:
        return v[:limit]
    return v


def _render(raw: Dict[str, Any]) -> Dict[str, Any]:
    exc: BaseException = raw["exc"]
    return {
        "ts": raw["ts"],
        "type": type(exc).__name__,
        "message": _truncate(str(exc)),
        "extras": {k: _truncate(v) for k, v in (raw["extras"] or {}).items()},
        "traceback": "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))[-4096:],
    }


def sentry_capture(exc: BaseException, *, extras: Optional[Dict[str, Any]] = None) -> None:
    """Record ``exc``.  Cheap on the hot path (the parser reports every failed
    message): the exception and extras are kept as-is in the bounded ring and
    rendered (message, truncation, traceback) only when read — or written at once
    when ``SMSGATE_ERROR_LOG`` asks for a durable log."""
    raw = {"ts": time.time(), "exc": exc, "extras": dict(extras) if extras else None}
    with _lock:
        _ring.append(raw)
    path = os.environ.get("SMSGATE_ERROR_LOG")
    if path:
        try:
            with open(path, "a", encoding="utf-8") as f:
                f.write(json.dumps(_render(raw), default=str, ensure_ascii=False) + "\n")
        except OSError:  # pragma: no cover
            pass
    sdk = _sdk
    if sdk is not None:  # pragma: no cover - SDK absent on the image
        with sdk.push_scope() as scope:
            for k, v in (extras or {}).items():
                scope.set_extra(k, v)
            sdk.capture_exception(exc)


def recent_errors(n: int = 100) -> List[Dict[str, Any]]:
    with _lock:
        raw = list(_ring)[-n:]
    return [_render(r) for r in raw]


def clear_errors() -> None:
    with _lock:
        _ring.clear()
