"""Persistence sinks: memory, SQL (PostgreSQL/SQLite), PocketBase REST."""
from .base import Sink  # noqa: F401
from .memory import MemorySink  # noqa: F401
