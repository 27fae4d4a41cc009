"""Multi-process HTTP gateway: N worker processes on one port with SO_REUSEPORT.

The reference scales its gateway by docker replicas (docker-compose.yml:65-79).
On one host, ``gateway --workers N`` starts N processes that each bind their own
listening socket to the same port with ``SO_REUSEPORT``: the kernel spreads new
connections over them by hash.  The sockets are created with ``IPPROTO_TCP``:
asyncio enables TCP_NODELAY on accepted connections only for such sockets, and
uvicorn's own ``workers=`` mode (proto 0) left every reply waiting on Nagle +
delayed ACK -- 4 of its workers served ~1 k req/s, these serve ~7.9 k
(``profiles/r03_ingest_bench.jsonl``).
Each worker builds the app from :func:`~smsgate_amd.services.gateway.default_app`
(its own bus client) and Prometheus counters are aggregated across workers
(``PROMETHEUS_MULTIPROC_DIR``, :func:`smsgate_amd.obs.metrics.render_latest`).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import shutil
import signal
import socket
import tempfile
import time
from typing import List

__all__ = ["serve_workers", "reuseport_socket"]


def reuseport_socket(host: str, port: int) -> socket.socket:
    # proto must say TCP: asyncio sets TCP_NODELAY on accepted connections only when
    # sock.proto == IPPROTO_TCP -- with proto 0 every reply waited out Nagle + delayed
    # ACK (~40 ms per request: 650 vs 1 900 req/s for one worker)
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.set_inheritable(True)
    return s


def _worker(host: str, port: int, log_level: str) -> None:
    import uvicorn

    from .gateway import default_app

    sock = reuseport_socket(host, port)
    cfg = uvicorn.Config(default_app(), log_level=log_level, access_log=False)
    uvicorn.Server(cfg).run(sockets=[sock])


def serve_workers(n: int, host: str, port: int, log_level: str = "warning") -> int:
    """Run ``n`` gateway processes on ``host:port`` until SIGTERM / SIGINT; returns 0."""
    own_dir = None
    if not os.environ.get("PROMETHEUS_MULTIPROC_DIR"):
        own_dir = os.environ["PROMETHEUS_MULTIPROC_DIR"] = tempfile.mkdtemp(prefix="smsgate-gw-metrics-")
    ctx = mp.get_context("spawn")
    procs: List[mp.Process] = []
    for i in range(n):
        p = ctx.Process(target=_worker, args=(host, port, log_level), name=f"gateway-{i}", daemon=False)
        p.start()
        procs.append(p)
    stop = {"flag": False}

    def on_signal(*_):
        stop["flag"] = True

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    try:
        while not stop["flag"] and all(p.is_alive() for p in procs):
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(10)
            if p.is_alive():
                p.kill()
        if own_dir:
            shutil.rmtree(own_dir, ignore_errors=True)
    return 0
