"""Writer-sink throughput (VERDICT r02 missing #4): rows/s of the sinks behind
``pb_writer`` (services/writer.py), one batch of ``--batch`` ParsedSMS per call.

* ``SqlSink`` on a SQLite file in WAL mode (the default store without Postgres):
  fresh inserts, then the same msg_ids again (``ON CONFLICT (msg_id) DO UPDATE``);
* ``PocketBaseSink`` against an in-process PocketBase fake whose every HTTP request
  costs ``--pb-latency-ms`` (a local PocketBase answers in ~1 ms): the reference's
  per-record path (GET by filter + POST/PATCH, 8 in flight) vs the batch API
  (``POST /api/batch``, 50 records per request).

Prints one JSON line.  (No Postgres and no PocketBase binary on the image: the
SQLite figure is a measurement, the PocketBase one is the client-side request
count and concurrency bound at the given per-request latency.)
"""
import argparse
import asyncio
import json
import os
import sys
import tempfile
import time
from datetime import datetime

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def _records(n, prefix):
    from smsgate_amd.models.domain import ParsedSMS

    return [ParsedSMS(msg_id=f"{prefix}{i}", device_id="d", sender="BANK", date=datetime(2025, 5, 6, 14, 23),
                      raw_body=f"APPROVED PURCHASE DB SALE: SHOP {i}, YEREVAN", txn_type="debit",
                      amount="52.00", currency="USD", card="0018", merchant=f"SHOP {i}", city="YEREVAN",
                      address="", balance="1842.74", parser_version="llm-0.2.0") for i in range(n)]


async def sql_bench(n, batch):
    from smsgate_amd.sinks.sql import SqlSink

    d = tempfile.mkdtemp(prefix="sinkbench-")
    sink = SqlSink(f"sqlite:///{d}/bench.sqlite")
    recs = _records(n, "m")
    out = {}
    for phase in ("insert", "update"):
        t0 = time.perf_counter()
        for i in range(0, n, batch):
            await sink.upsert_many(recs[i:i + batch])
        out[f"{phase}_rows_per_s"] = round(n / (time.perf_counter() - t0), 1)
    out["rows"] = sink.count()
    await sink.close()
    return out


async def pb_bench(n, batch, latency_ms):
    import httpx
    from fakes import FakePocketBase

    from smsgate_amd.sinks.pocketbase import PocketBaseClient, PocketBaseSink

    res = {}
    for mode in ("per_record", "batch_api"):
        fake = FakePocketBase(batch_enabled=mode == "batch_api")

        class Slow(httpx.AsyncBaseTransport):
            async def handle_async_request(self, req):
                await asyncio.sleep(latency_ms / 1000.0)
                await req.aread()
                return fake.handle(req)

        c = PocketBaseClient(base_url="http://pb", transport=Slow())
        sink = PocketBaseSink(c, batch=50 if mode == "batch_api" else 1)
        recs = _records(n, "p")
        t0 = time.perf_counter()
        for i in range(0, n, batch):
            await sink.upsert_many(recs[i:i + batch])
        dt = time.perf_counter() - t0
        await c.close()
        res[mode] = {"rows_per_s": round(n / dt, 1), "requests": len(fake.calls),
                     "requests_per_row": round(len(fake.calls) / n, 3), "stored": len(fake.cols.get("sms_data", []))}
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=50000)
    p.add_argument("--pb-rows", type=int, default=5000)
    p.add_argument("--batch", type=int, default=512)
    p.add_argument("--pb-latency-ms", type=float, default=1.0)
    a = p.parse_args()
    out = {"bench": "writer_sinks", "batch": a.batch, "sqlite_wal": asyncio.run(sql_bench(a.rows, a.batch)),
           "pocketbase": asyncio.run(pb_bench(a.pb_rows, a.batch, a.pb_latency_ms)),
           "pb_latency_ms": a.pb_latency_ms}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
