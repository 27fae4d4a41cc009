"""Blocking client for the broker's msgpack protocol (``bus/server.py`` / ``smsgate-busd``).

For callers without an event loop — the GPU rank process of the benchmark polls
consumer state between engine steps with it.  Requests are synchronous
(``[op, rid, *args]`` → ``[rid, ok, result]``); nothing is pipelined.
"""
from __future__ import annotations

import itertools
import socket
import struct
from typing import Any, Dict
from urllib.parse import urlparse

import msgpack

from .base import BusError

__all__ = ["SyncBusClient"]

_LEN = struct.Struct("<I")


class SyncBusClient:
    """``dsn``: one broker (``unix://`` / ``tcp://``) or a ``sharded+...`` list
    (:mod:`.sharded`): then a durable is looked up on the shard owning it."""

    def __new__(cls, dsn: str, timeout: float = 10.0):
        if dsn.startswith("sharded+"):
            return _SyncSharded([d for d in dsn[len("sharded+"):].split(",") if d], timeout)
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
                raise BusError("bus connection closed")
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

    def consumer_info(self, stream: str, durable: str) -> Dict[str, Any]:
        return self.call("consumer_info", stream, durable)

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class _SyncSharded:
    def __init__(self, dsns, timeout: float) -> None:
        self.members = [SyncBusClient(d, timeout) for d in dsns]

    def ensure_stream(self) -> None:
        for m in self.members:
            m.ensure_stream()

    def subscribe(self, subject: str, durable: str, **opts: Any) -> str:
        from .sharded import shard_of

        return self.members[shard_of(subject, len(self.members))].subscribe(subject, durable, **opts)

    def consumer_info(self, stream: str, durable: str) -> Dict[str, Any]:
        err: Exception = BusError(f"consumer {durable!r} not found on any shard")
        for m in self.members:
            try:
                return m.consumer_info(stream, durable)
            except BusError as exc:
                err = exc
        raise err

    def close(self) -> None:
        for m in self.members:
            m.close()
