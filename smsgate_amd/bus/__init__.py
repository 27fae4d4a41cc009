"""Durable subject bus (the reference's NATS JetStream role).

:func:`connect` maps a DSN to a backend:

* ``memory://`` / ``memory://<name>`` — in-process :class:`MemoryBus`
  (one shared instance per name and event loop);
* ``file:///path/to/dir`` — in-process engine with a crash-safe segment log
  (single process owns the directory);
* ``tcp://host:port`` / ``unix:///path.sock`` — :class:`RemoteBus` client of a
  ``python -m smsgate_amd bus-server`` broker process;
* ``nats://host:port`` — :class:`~.nats_client.NatsBus`: the NATS wire protocol +
  JetStream API (no nats-py needed), against a real ``nats-server`` or our broker's
  NATS front-end (``bus-server --nats-listen``);
* ``sharded+<dsn>,<dsn>...`` — :class:`~.sharded.ShardedBus`: several brokers as
  one bus, sharded by subject (``sms.raw`` on the first).
"""
from __future__ import annotations

import asyncio
from typing import Dict, Optional, Tuple
from urllib.parse import urlparse

from .base import (  # noqa: F401
    ALL_SUBJECTS,
    STREAM_NAME,
    SUBJECT_CATEGORIZED,
    SUBJECT_FAILED,
    SUBJECT_PARSED,
    SUBJECT_PROCESSING,
    SUBJECT_RAW,
    Bus,
    BusError,
    BusUnavailable,
    ConsumerConfig,
    ConsumerInfo,
    DeliverPolicy,
    Msg,
    PubAck,
    StreamConfig,
    StreamInfo,
    Subscription,
    default_stream_config,
    subject_matches,
)
from .engine import Engine  # noqa: F401
from .memory import MemoryBus  # noqa: F401

__all__ = [
    "connect",
    "reset_connections",
    "Bus",
    "MemoryBus",
    "Engine",
    "SUBJECT_RAW",
    "SUBJECT_PARSED",
    "SUBJECT_PROCESSING",
    "SUBJECT_FAILED",
    "SUBJECT_CATEGORIZED",
    "STREAM_NAME",
]

_shared: Dict[Tuple[str, int], Bus] = {}
_locks: Dict[int, asyncio.Lock] = {}


def reset_connections() -> None:
    """Forget cached connections (tests)."""
    _shared.clear()
    _locks.clear()


async def _open(dsn: str, max_age: float) -> Bus:
    if dsn.startswith("sharded+"):
        from .sharded import ShardedBus

        return await ShardedBus.connect([d for d in dsn[len("sharded+"):].split(",") if d], max_age)
    u = urlparse(dsn)
    scheme = u.scheme or "memory"
    if scheme == "memory":
        return MemoryBus(max_age=max_age)
    if scheme == "file":
        from .filelog import open_file_bus

        return await open_file_bus(u.path or u.netloc, max_age=max_age)
    if scheme in ("tcp", "unix"):
        from .client import RemoteBus

        return await RemoteBus.connect(dsn)
    if scheme == "nats":
        from .nats_client import connect_nats

        return await connect_nats(dsn)
    if scheme in ("redis", "rediss"):
        # The reference's stale default (config.py:27) — treat as in-process.
        return MemoryBus(max_age=max_age)
    raise BusError(f"unsupported bus DSN {dsn!r}")


async def connect(dsn: Optional[str] = None, *, shared: bool = True,
                  max_age: float = 3 * 24 * 3600.0) -> Bus:
    """Open (or reuse, when ``shared``) a bus connection — the reference's
    ``get_nats_connection`` singleton (nats_utils.py:38-47), made safe for
    concurrent first calls with a per-loop lock.
    """
    if dsn is None:
        from ..config import get_settings

        dsn = get_settings().nats_dsn
    if not shared:
        return await _open(dsn, max_age)
    loop_id = id(asyncio.get_running_loop())
    key = (dsn, loop_id)
    bus = _shared.get(key)
    if bus is not None:
        return bus
    lock = _locks.setdefault(loop_id, asyncio.Lock())
    async with lock:
        bus = _shared.get(key)
        if bus is None:
            bus = _shared[key] = await _open(dsn, max_age)
    return bus
