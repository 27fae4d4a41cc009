"""Native (host C++) runtime components.

* ``smsgate-busd`` (``csrc/busd.cpp`` + ``engine.hpp`` + ``mpack.hpp``): the
  durable bus broker in C++ — the role the reference fills with an external
  NATS server (docker-compose.yml:15-27).  It speaks the
  same msgpack protocol as ``python -m smsgate_amd bus-server`` (so
  :class:`~smsgate_amd.bus.client.RemoteBus` works unchanged) and writes the
  same CRC-framed journal as :mod:`smsgate_amd.bus.filelog` (either broker
  recovers the other's data directory).  One epoll loop, group-committed
  journal writes, long-poll fetch waiters.  ``nats_listen`` adds the NATS client
  protocol + JetStream API front-end (the subset :mod:`smsgate_amd.bus.nats_server`
  serves) on the same engine, so nats-py style clients reach the fast broker.
  ``http_listen`` adds native HTTP ingestion (``csrc/http_ingest.hpp``): the
  gateway's ``POST /sms/raw`` / ``/sms/raw/batch`` contract, ``/health``,
  ``/metrics``, stored straight into ``sms.raw`` by the broker's own loop.

Build: ``python -m smsgate_amd.native.build`` (in-tree, ``_bin/``).
"""
from __future__ import annotations

import os
import signal
import subprocess
import time
from pathlib import Path
from typing import List, Optional

from .build import BUSD, BUSD_SAN

__all__ = ["BUSD", "BUSD_SAN", "available", "NativeBroker", "spawn_busd"]


def available(binary: Path = BUSD) -> bool:
    return binary.exists() and os.access(binary, os.X_OK)


class NativeBroker:
    """A running ``smsgate-busd`` child process."""

    def __init__(self, proc: subprocess.Popen, listens: List[str], tcp_port: Optional[int],
                 nats_port: Optional[int] = None, http_port: Optional[int] = None) -> None:
        self.proc = proc
        self.listens = listens
        self.tcp_port = tcp_port
        self.nats_port = nats_port
        self.http_port = http_port

    @property
    def pid(self) -> int:
        return self.proc.pid

    def alive(self) -> bool:
        return self.proc.poll() is None

    def stop(self, timeout: float = 10.0) -> int:
        """Graceful stop (SIGTERM: flush + fsync the journal); returns the exit code."""
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        return self.proc.returncode

    def kill(self) -> None:
        """Crash it (SIGKILL) — for recovery tests."""
        if self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()

    async def close(self) -> None:  # same shape as BusServer.close()
        self.stop()


def spawn_busd(listen: str | List[str], data_dir: Optional[str] = None, *, max_age: float = 3 * 24 * 3600.0,
               fsync: str = "interval", fsync_interval_s: float = 0.05, compact_bytes: Optional[int] = None,
               ready_timeout: float = 20.0, binary: Optional[Path] = None, stderr=None,
               die_with_parent: bool = True, nats_listen: Optional[str] = None,
               http_listen: Optional[str] = None) -> NativeBroker:
    """Start the native broker and wait until it listens.

    ``listen`` takes ``tcp://host:port`` (port 0 = pick one, see
    :attr:`NativeBroker.tcp_port`) and/or ``unix:///path`` URLs.  With
    ``die_with_parent`` the broker gets SIGTERM when the starting process dies
    (no orphaned broker after a crashed benchmark or test).
    """
    binary = Path(binary or BUSD)
    if not available(binary):
        raise RuntimeError(f"{binary} is not built (python -m smsgate_amd.native.build)")
    listens = [listen] if isinstance(listen, str) else list(listen)
    cmd = [str(binary)]
    for u in listens:
        cmd += ["--listen", u]
    if nats_listen:
        cmd += ["--nats-listen", nats_listen]
    if http_listen:
        cmd += ["--http-listen", http_listen]
    if data_dir:
        cmd += ["--data", str(data_dir)]
    cmd += ["--max-age", repr(float(max_age)), "--fsync", fsync, "--fsync-interval", repr(float(fsync_interval_s))]
    if compact_bytes is not None:
        cmd += ["--compact-bytes", str(int(compact_bytes))]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stdin=subprocess.DEVNULL, stderr=stderr,
                            preexec_fn=_pdeathsig if die_with_parent else None)
    t_end = time.monotonic() + ready_timeout
    line = b""
    while time.monotonic() < t_end:
        line = proc.stdout.readline()  # type: ignore[union-attr]
        if line or proc.poll() is not None:
            break
    if not line.startswith(b"READY"):
        proc.kill()
        raise RuntimeError(f"smsgate-busd failed to start (exit {proc.poll()}): {line!r}")
    parts = line.split()
    tok = parts[1].decode()
    extra = {parts[k].decode(): int(parts[k + 1]) for k in range(2, len(parts) - 1, 2)}  # "NATS p", "HTTP p"
    return NativeBroker(proc, listens, None if tok == "-" else int(tok), extra.get("NATS"), extra.get("HTTP"))


def _pdeathsig() -> None:  # runs in the child between fork and exec
    import ctypes

    ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG

