"""Blocking client for the broker's msgpack protocol (``bus/server.py`` / ``smsgate-busd``).

For callers without an event loop — the GPU rank process of the benchmark polls
consumer state between engine steps with it.  Requests are synchronous
(``[op, rid, *args]`` → ``[rid, ok, result]``); nothing is pipelined.
"""
from __future__ import annotations

import itertools
import socket
import struct
from typing import Any, Dict, List, Optional
from urllib.parse import urlparse

import msgpack

from .base import BusError, BusUnavailable

__all__ = ["SyncBusClient"]

_LEN = struct.Struct("<I")


class SyncBusClient:
    """``dsn``: one broker (``unix://`` / ``tcp://``) or a ``sharded+...`` list
    (:mod:`.sharded`): then a durable is looked up on the shard owning it."""

    def __new__(cls, dsn: str, timeout: float = 10.0):
        if dsn.startswith("sharded+"):
            return _SyncSharded(dsn[len("sharded+"):], timeout)
        return super().__new__(cls)

    def __init__(self, dsn: str, timeout: float = 10.0) -> None:
        u = urlparse(dsn)
        if u.scheme == "unix":
            self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            self.sock.settimeout(timeout)
            self.sock.connect(u.path)
        else:
            self.sock = socket.create_connection((u.hostname or "127.0.0.1", u.port or 4222), timeout=timeout)
        self._ids = itertools.count(1)

    def _read(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise BusUnavailable("bus connection closed")
            buf += chunk
        return bytes(buf)

    def call(self, op: str, *args: Any) -> Any:
        rid = next(self._ids)
        body = msgpack.packb([op, rid, *args], use_bin_type=True)
        self.sock.sendall(_LEN.pack(len(body)) + body)
        while True:
            (n,) = _LEN.unpack(self._read(4))
            r_id, ok, res = msgpack.unpackb(self._read(n), raw=False, strict_map_key=False)
            if r_id == rid:
                if not ok:
                    raise BusError(res)
                return res

    def ensure_stream(self) -> None:
        self.call("ensure_stream", None)

    def subscribe(self, subject: str, durable: str, **opts: Any) -> str:
        return self.call("subscribe", subject, durable, opts)

    def consumer_info(self, stream: str, durable: str, subject: Optional[str] = None) -> Dict[str, Any]:
        return self.call("consumer_info", stream, durable)

    def stream_info(self, stream: str = "SMS") -> Dict[str, Any]:
        return self.call("stream_info", stream)

    def member_stats(self, stream: str = "SMS") -> List[Dict[str, Any]]:
        """One broker: its message count (the sharded view reports every member)."""
        return [{"subjects": ["*"], "messages": int(self.stream_info(stream).get("messages", 0))}]

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class _SyncSharded:
    """Blocking view of a ``sharded+`` bus (positional or pinned/partitioned layout,
    :mod:`.sharded`): a durable of a partitioned subject exists on every partition
    and its consumer_info is the sum over them."""

    def __init__(self, spec: str, timeout: float) -> None:
        from .sharded import Router, parse_members

        dsns, pins, default = parse_members(spec)
        self.members = [SyncBusClient(d, timeout) for d in dsns]
        self.router = Router(len(dsns), pins, default)

    def ensure_stream(self) -> None:
        for m in self.members:
            m.ensure_stream()

    def subscribe(self, subject: str, durable: str, **opts: Any) -> str:
        names = [self.members[k].subscribe(subject, durable, **opts) for k in self.router.members(subject)]
        return names[0]

    def consumer_info(self, stream: str, durable: str, subject: Optional[str] = None) -> Dict[str, Any]:
        """Summed over the members; with ``subject`` only the members that subject is
        routed to are asked (one round trip per partition instead of one per broker)."""
        found = []
        members = self.members if subject is None else [self.members[k] for k in self.router.members(subject)]
        for m in members:
            try:
                found.append(m.consumer_info(stream, durable))
            except BusError:
                continue
        if not found:
            raise BusError(f"consumer {durable!r} not found on any shard")
        if len(found) == 1:
            return found[0]
        out = dict(found[0])
        for k in ("num_pending", "num_ack_pending", "num_redelivered", "num_waiting"):
            if k in out:
                out[k] = sum(f.get(k, 0) for f in found)
        return out

    def member_stats(self, stream: str = "SMS") -> List[Dict[str, Any]]:
        """Per broker: the subjects pinned to it and the messages its stream holds (the
        node layout check: every partition of sms.raw carries traffic)."""
        pinned: Dict[int, List[str]] = {}
        for subj, idx in self.router.pins.items():
            for k in idx:
                pinned.setdefault(k, []).append(subj)
        return [{"subjects": pinned.get(k, ["*"]), "messages": int(m.stream_info(stream).get("messages", 0))}
                for k, m in enumerate(self.members)]

    def close(self) -> None:
        for m in self.members:
            m.close()
