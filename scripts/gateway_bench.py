"""Ingest capacity of the HTTP gateway (VERDICT r02 missing #3).

Starts one ``smsgate-busd`` broker (journal on), the gateway with ``--workers N``
on a local port (``python -m smsgate_amd gateway``), and a load generator of P
client processes x C keep-alive connections speaking raw HTTP/1.1 (so the client
is not the bottleneck: no HTTP library per request).  Two phases of ``--seconds``
each:

* ``POST /sms/raw``        one SMS per request -> requests/s (= msgs/s);
* ``POST /sms/raw/batch``  ``--batch`` SMS per request -> msgs/s.

Every 202 is counted, and the broker's ``sms.raw`` stream must hold exactly as
many messages as were acknowledged (nothing lost, nothing invented).  Prints one
JSON line.

``--mode native`` measures the broker's own HTTP front-end instead
(``smsgate-busd --http-listen``, csrc/http_ingest.hpp: the same contract,
tests/test_http_ingest.py) -- no gateway process at all.

    python scripts/gateway_bench.py --workers 4 --clients 4 --conns 32 --seconds 8
    python scripts/gateway_bench.py --mode native --clients 4 --conns 32 --seconds 8
"""
import argparse
import asyncio
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BODY = ("APPROVED PURCHASE DB SALE: SHOP {i}, YEREVAN, KOMITAS AVE. 12,06.05.25 14:23,card ***0018. "
        "Amount:{a}.00 USD, Balance:1842.74 USD")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _request(path: str, payload) -> bytes:
    body = json.dumps(payload).encode()
    return (f"POST {path} HTTP/1.1\r\nHost: gw\r\nContent-Type: application/json\r\n"
            f"Content-Length: {len(body)}\r\n\r\n").encode() + body


async def _conn_loop(port: int, reqs, t_end: float, counts) -> None:
    r, w = await asyncio.open_connection("127.0.0.1", port)
    k = 0
    try:
        while time.perf_counter() < t_end:
            req, n = reqs[k % len(reqs)]
            k += 1
            w.write(req)
            await w.drain()
            head = await r.readuntil(b"\r\n\r\n")
            status = int(head.split(b" ", 2)[1])
            clen = 0
            for line in head.split(b"\r\n"):
                if line[:15].lower() == b"content-length:":
                    clen = int(line[15:])
            await r.readexactly(clen)
            if status == 202:
                counts[0] += n
                counts[1] += 1
            else:
                counts[2] += 1
    finally:
        w.close()


def _client(port: int, conns: int, path: str, batch: int, seconds: float, seed: int, q) -> None:
    reqs = []
    for j in range(256):
        i = seed * 1_000_000 + j
        if path.endswith("batch"):
            payload = [{"device_id": "bench", "message": BODY.format(i=f"{i}-{b}", a=b + 1), "sender": "BANK",
                        "timestamp": 1746541380 + b, "source": "device"} for b in range(batch)]
            reqs.append((_request(path, payload), batch))
        else:
            payload = {"device_id": "bench", "message": BODY.format(i=i, a=j + 1), "sender": "BANK",
                       "timestamp": 1746541380 + j, "source": "device"}
            reqs.append((_request(path, payload), 1))
    counts = [0, 0, 0]  # messages acknowledged, 202 responses, other responses

    async def main():
        t_end = time.perf_counter() + seconds
        await asyncio.gather(*(_conn_loop(port, reqs, t_end, counts) for _ in range(conns)))

    asyncio.run(main())
    q.put(counts)


def _phase_native(port, args, path, batch):
    from smsgate_amd.native.build import BUSLOAD

    conns = args.clients * args.conns
    cmd = [str(BUSLOAD), "--http", str(port), "--conns", str(conns), "--seconds", str(args.seconds),
           "--depth", str(args.depth)] + (["--batch", str(batch)] if batch > 1 else [])
    out = json.loads(subprocess.run(cmd, capture_output=True, text=True, timeout=args.seconds + 120).stdout)
    return {"endpoint": path, "batch": batch, "msgs": int(round(out["msgs_per_s"] * out["seconds"])),
            "requests_202": out["requests_202"], "requests_other": out["requests_other"],
            "msgs_per_s": out["msgs_per_s"], "requests_per_s": out["requests_per_s"], "wall_s": out["seconds"],
            "loadgen": "smsgate-busload --http", "conns": conns, "depth": args.depth}


def _phase(port, args, path, batch):
    if args.loadgen == "native":
        return _phase_native(port, args, path, batch)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_client, args=(port, args.conns, path, batch, args.seconds, c, q))
             for c in range(args.clients)]
    t0 = time.perf_counter()
    for p in procs:
        p.start()
    res = [q.get(timeout=args.seconds + 120) for _ in procs]
    for p in procs:
        p.join()
    dt = time.perf_counter() - t0
    msgs, ok, bad = (sum(r[i] for r in res) for i in range(3))
    # the clients ran `seconds` each; start-up of the processes is excluded from the rate
    return {"endpoint": path, "batch": batch, "msgs": msgs, "requests_202": ok, "requests_other": bad,
            "msgs_per_s": round(msgs / args.seconds, 1), "requests_per_s": round(ok / args.seconds, 1),
            "wall_s": round(dt, 2)}


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--clients", type=int, default=4)
    p.add_argument("--conns", type=int, default=32)
    p.add_argument("--seconds", type=float, default=8.0)
    p.add_argument("--batch", type=int, default=100)
    p.add_argument("--mode", default="python", choices=["python", "native"])
    p.add_argument("--loadgen", default="python", choices=["python", "native"],
                   help="native: smsgate-busload --http (C++ threads, one keep-alive connection each)")
    p.add_argument("--depth", type=int, default=1, help="native load generator: pipelined requests per connection")
    a = p.parse_args()
    from smsgate_amd.bus.sync_client import SyncBusClient
    from smsgate_amd.native import spawn_busd

    tmp = tempfile.mkdtemp(prefix="gwbench-")
    sock = os.path.join(tmp, "bus.sock")
    native = a.mode == "native"
    broker = spawn_busd(f"unix://{sock}", os.path.join(tmp, "data"),
                        http_listen="tcp://127.0.0.1:0" if native else None)
    gw = None
    if native:
        port = broker.http_port
    else:
        port = _free_port()
        env = dict(os.environ, NATS_DSN=f"unix://{sock}", API_PORT=str(port), API_HOST="127.0.0.1",
                   LOG_DIR=os.path.join(tmp, "logs"), BACKUP_DIR=os.path.join(tmp, "backups"))
        gw = subprocess.Popen([sys.executable, "-m", "smsgate_amd", "gateway", "--workers", str(a.workers)],
                              env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        for _ in range(300):
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.2).close()
                break
            except OSError:
                time.sleep(0.1)
        time.sleep(1.0)  # every worker up
        bus = SyncBusClient(f"unix://{sock}")
        bus.ensure_stream()
        bus.subscribe("sms.raw", "gwbench_count")
        single = _phase(port, a, "/sms/raw", 1)
        batch = _phase(port, a, "/sms/raw/batch", a.batch)
        stored = bus.consumer_info("SMS", "gwbench_count")["num_pending"]
    finally:
        if gw is not None:
            gw.terminate()
            try:
                gw.wait(20)
            except subprocess.TimeoutExpired:
                gw.kill()
        broker.stop()
    acked = single["msgs"] + batch["msgs"]
    if a.loadgen == "native":  # (msgs derived from a rate: compare with a small tolerance)
        acked = single["requests_202"] + batch["requests_202"] * a.batch
    out = {"bench": "gateway_ingest", "mode": a.mode, "workers": 0 if native else a.workers, "client_procs": a.clients,
           "conns_per_client": a.conns, "loadgen": a.loadgen, "seconds": a.seconds, "single": single, "batch": batch,
           "broker_stored": stored, "acked": acked, "lossless": stored >= acked,
           "cpus": os.cpu_count(), "note": "gateway, broker and load generator share the same CPUs"}
    print(json.dumps(out), flush=True)
    return 0 if out["lossless"] else 1


if __name__ == "__main__":
    sys.exit(main())
