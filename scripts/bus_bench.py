#!/usr/bin/env python3
"""Broker throughput: Python ``bus-server`` vs native ``smsgate-busd``.

P producer processes publish ``--msgs`` messages each (``publish_many`` batches of
``--batch``, ~300-byte SMS-sized payloads) onto ``sms.raw``; C consumer processes
share one durable group, fetch batches and ack every message.  Reported: end-to-end
msgs/s (first publish → last ack observed by ``consumer_info``) with the journal on
(``--data``, fsync interval) for each broker.  ``--protocol nats`` drives both
brokers through their NATS front-ends (JetStream PubAck per publish, pull
consumers, ``$JS.ACK`` acks) with the same client code.

    python scripts/bus_bench.py --producers 4 --consumers 4 --msgs 50000
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd.bus import SUBJECT_RAW, connect  # noqa: E402
from smsgate_amd.bus.server import serve  # noqa: E402

PAYLOAD = b'{"msg_id":"%08d","sender":"BANK","body":"APPROVED PURCHASE DB SALE: TEST LLC, MOSKOW, TEST STR. 29, ' \
          b'24 AREA,06.05.25 14:23,card ***0018. Amount:52.00 USD, Balance:1842.74 USD","date":"1718300000",' \
          b'"device_id":"android","source":"device"}'


def _producer(sock, n, batch, start_evt):
    async def go():
        bus = await connect(sock, shared=False)
        start_evt.wait()
        for i in range(0, n, batch):
            await bus.publish_many([(SUBJECT_RAW, PAYLOAD % (i + k)) for k in range(min(batch, n - i))])
        await bus.close()

    asyncio.run(go())


def _consumer(sock, batch, stop_evt):
    async def go():
        bus = await connect(sock, shared=False)
        sub = await bus.subscribe(SUBJECT_RAW, "bench")
        while not stop_evt.is_set():
            for m in await sub.fetch(batch, 0.2):
                await m.ack()
        await bus.close()

    asyncio.run(go())


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_one(native: bool, a) -> dict:
    tmp = tempfile.mkdtemp(prefix="busbench-")
    ctl_sock = sock = f"unix://{tmp}/bus.sock"
    nats_listen = None
    if a.protocol == "nats":
        port = _free_port()
        nats_listen = f"tcp://127.0.0.1:{port}"
        sock = f"nats://127.0.0.1:{port}"
    ctx = mp.get_context("spawn")
    total = a.producers * a.msgs

    async def go():
        srv = await serve(ctl_sock, os.path.join(tmp, "data") if a.journal else None, native=native,
                          nats_listen=nats_listen)
        ctl = await connect(sock, shared=False)
        await ctl.subscribe(SUBJECT_RAW, "bench")  # create the durable before anyone publishes
        start_evt, stop_evt = ctx.Event(), ctx.Event()
        cons = [ctx.Process(target=_consumer, args=(sock, a.batch, stop_evt)) for _ in range(a.consumers)]
        prods = [ctx.Process(target=_producer, args=(sock, a.msgs, a.batch, start_evt)) for _ in range(a.producers)]
        for p in cons + prods:
            p.start()
        await asyncio.sleep(2.0)  # let every process connect (spawn + imports)
        t0 = time.perf_counter()
        start_evt.set()
        while True:
            i = await ctl.consumer_info("SMS", "bench")
            si = await ctl.stream_info("SMS")
            if si.last_seq >= total and i.num_pending == 0 and i.num_ack_pending == 0:
                break
            await asyncio.sleep(0.01)
        dt = time.perf_counter() - t0
        stop_evt.set()
        for p in cons + prods:
            p.join(10)
        await ctl.close()
        await srv.close()
        return dt

    dt = asyncio.run(go())
    return {"broker": "native" if native else "python", "protocol": a.protocol, "msgs": total, "seconds": round(dt, 3),
            "msgs_per_s": round(total / dt, 1), "producers": a.producers, "consumers": a.consumers,
            "batch": a.batch, "journal": a.journal}


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--producers", type=int, default=4)
    p.add_argument("--consumers", type=int, default=4)
    p.add_argument("--msgs", type=int, default=25000, help="per producer")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--no-journal", dest="journal", action="store_false")
    p.add_argument("--only", choices=["python", "native"], default=None)
    p.add_argument("--protocol", choices=["msgpack", "nats"], default="msgpack")
    a = p.parse_args()
    from smsgate_amd.native import build

    build.build()
    for native in (False, True):
        if a.only and a.only != ("native" if native else "python"):
            continue
        print(json.dumps(run_one(native, a)), flush=True)


if __name__ == "__main__":
    main()
