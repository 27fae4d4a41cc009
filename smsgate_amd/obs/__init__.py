"""Observability: Prometheus metrics, error capture, tracing spans, logging."""
from .errors import clear_errors, init_sentry, recent_errors, sentry_capture  # noqa: F401
from .tracing import start_span, start_transaction, tracer  # noqa: F401
