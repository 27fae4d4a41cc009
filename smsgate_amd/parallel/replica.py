"""One data-parallel replica per MI355X: a GPU engine process + K CPU parser processes.

The reference scales by running more ``parser_worker`` containers in one
durable consumer group (worker.py:199-202). Here one replica per GPU is the
unit of scale-out; inside a replica the work is split by resource:

* the **rank process** (one per GPU under torchrun) owns the GPU — the
  extraction engine with its hipGraph-captured decode — and serves token-id
  batches to its workers (:class:`~smsgate_amd.serving.remote.EngineServer`);
  across ranks it joins a ``torch.distributed`` group over RCCL for barriers
  and metric reductions (no per-message collectives: replicas are independent
  competing consumers, the right call for a model that fits one GPU —
  SURVEY.md §5.8);
* **K parser processes** run the CPU side of the parser stage (bus I/O,
  JSON, validation, tokenisation, post-processing, DLQ routing), each with its
  own interpreter so no GIL is shared with the GPU feeder.

Parser processes are spawned *before* the rank process touches the GPU.
"""
from __future__ import annotations

import asyncio
import multiprocessing as mp
import os
import time
from multiprocessing.connection import Connection
from typing import Any, Dict, List, Optional, Sequence, Tuple

__all__ = ["spawn_parser_workers", "parser_worker_main", "Coordinator"]


def spawn_parser_workers(n: int, rank: int, cfg: Dict[str, Any]) -> Tuple[List[Any], List[Connection]]:
    """Start ``n`` parser processes (spawn context, GPU hidden); returns (procs, conns)."""
    ctx = mp.get_context("spawn")
    procs, conns = [], []
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                            "RAYON_NUM_THREADS", "OMP_NUM_THREADS")}
    try:
        # parser processes never touch the GPU; hide it so an accidental CUDA call fails fast
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
        # the tokenizer's Rust thread pool defaults to one thread per CPU of the whole
        # machine in EVERY worker (K workers per GPU x 8 GPUs); give each a small share
        threads = int(cfg.get("worker_threads", 2))
        if threads > 0 and saved["RAYON_NUM_THREADS"] is None:
            os.environ["RAYON_NUM_THREADS"] = str(threads)
        os.environ["OMP_NUM_THREADS"] = "1"
        for w in range(n):
            a, b = ctx.Pipe(duplex=True)
            p = ctx.Process(target=parser_worker_main, args=(b, rank, w, cfg), name=f"parser-r{rank}-w{w}",
                            daemon=True)
            p.start()
            b.close()
            procs.append(p)
            conns.append(a)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return procs, conns


def _payload_bytes(n: int, seed: int, vocab_name: str = "heldout", traffic: str = "mixed") -> List[bytes]:
    """Synthetic phone posts (the gateway's ``RawSMSPayload``); ``vocab_name``
    picks the merchant / city vocabulary (held-out = never seen in training),
    ``traffic`` the preset mix of SMS layouts / kinds (utils.synth.TRAFFIC)."""
    from ..services.gateway import RawSMSPayload
    from ..utils.synth import generate_traffic

    out = []
    for s in generate_traffic(n, seed=seed, vocab_name=vocab_name, traffic=traffic):
        p = RawSMSPayload(device_id="bench", message=s.body, sender="BANK", timestamp=s.timestamp, source="device")
        out.append(p)
    return out  # type: ignore[return-value]


def parser_worker_main(conn: Connection, rank: int, widx: int, cfg: Dict[str, Any]) -> None:
    """Entry point of a parser process (bench/serving harness).  ``cfg["nice"]`` > 0
    lowers its CPU priority: on a node where the parser processes and the rank process
    share cores, the rank process (it feeds the GPU) wins a contended core."""
    if int(cfg.get("nice", 0)) > 0:
        os.nice(int(cfg["nice"]))
    asyncio.run(_worker_async(conn, rank, widx, cfg))


async def _worker_async(conn: Connection, rank: int, widx: int, cfg: Dict[str, Any]) -> None:
    from ..bus import SUBJECT_RAW, MemoryBus
    from ..parse.backends.local_llm import RemoteLLMBackend
    from ..parse.pipeline import ParsePipeline
    from ..serving.remote import RemoteEngineClient
    from ..parse.fastpath import raw_wires  # the gateway role's payload -> sms.raw bytes (native)
    from ..services.parser import ParserWorker
    from ..services.writer import WriterService
    from ..sinks.memory import MemorySink

    from ..bus import connect

    client = RemoteEngineClient(conn, max_body_tokens=cfg.get("max_body_tokens", 128))
    dsn = cfg.get("bus")
    # shared broker: every parser process of every GPU is ONE competing group on sms.raw
    # (worker.py:199-202 semantics) and every writer one group on sms.parsed;
    # memory: each process runs its own in-process bus (isolated partitions)
    bus = await connect(dsn, shared=False) if dsn else MemoryBus()
    backend = RemoteLLMBackend(client, max_batch=cfg.get("batch", 512))
    worker = ParserWorker(bus, ParsePipeline(backend), batch=cfg.get("batch", 512),
                          concurrency=cfg.get("concurrency", 4), stats_interval=0)
    if dsn:
        worker.stage.max_ack_pending = 1 << 22  # all replicas' batches in flight at once
    # pb_writer on sms.parsed with an in-memory sink (BASELINE config #1: "... -> in-memory
    # sink"), or a real SqlSink: one SQLite WAL file per parser process (--sink sqlite)
    if cfg.get("sink", "memory") == "sqlite":
        from ..sinks.sql import SqlSink

        sink = SqlSink(f"sqlite:///{cfg['sink_dir']}/sink-r{rank}-w{widx}.db")
    else:
        sink = MemorySink()
    writer = WriterService(bus, [sink], batch=cfg.get("writer_batch", 512), stats_interval=0)
    if dsn:
        writer.stage.max_ack_pending = 1 << 22
    await worker.start()
    await writer.start()
    client.send_control({"event": "ready", "w": widx})
    prepared: List[List[Any]] = []
    # cProfile of the phases the coordinator marks as profiled (bench.py --profile-cpu DIR:
    # the timed bus phase only -- not the warm-up or the HTTP phase); prof_msgs counts the
    # messages this process parsed while it was on, the per-message denominator
    prof = None
    prof_msgs = 0
    if cfg.get("profile_dir"):
        if cfg.get("profile_mode", "sample") == "sample":  # CPU-time sampling (utils/sampler.py)
            from ..utils.sampler import CpuSampler

            prof = CpuSampler()
            prof.enable, prof.disable = prof.start, prof.stop
        else:
            import cProfile

            prof = cProfile.Profile()
    while True:
        cmd = await asyncio.to_thread(client.control.get)
        if cmd is None or cmd.get("cmd") == "quit":
            break
        if cmd["cmd"] == "prepare":
            n = int(cmd["n"])
            prepared = [_payload_bytes(n, seed, cfg.get("vocab", "heldout"), cfg.get("traffic", "mixed"))
                        for seed in cmd["seeds"]]
            # the phase's counters start HERE, before any process is told to go: with a
            # shared broker the parser and writer groups span every process, so a process
            # that reads its "go" late has already parsed / written messages other
            # processes published, and a snapshot taken at "go" would drop them
            c0 = dict(worker.counts)
            w0 = (writer.stage.processed, writer.ok, writer.skipped, writer.fail)
            base = worker.stage.processed
            client.send_control({"event": "prepared", "w": widx})
        elif cmd["cmd"] == "go":
            profiling = prof is not None and bool(cmd.get("profile"))
            if profiling:
                prof.enable()
            t0 = time.perf_counter()

            async def publish(i: int) -> None:
                # gateway ingestion in chunks that yield to the parser stage, so parsing
                # (and the GPU) start after the first chunk, not after whole steps
                chunk = 256
                msgs = prepared[i]
                for c in range(0, len(msgs), chunk):
                    items = [(SUBJECT_RAW, w) for w in raw_wires(msgs[c:c + chunk])]
                    await bus.publish_many(items)
                    await asyncio.sleep(0)

            nsteps = len(prepared)
            if dsn:
                # shared broker: ingest everything (the gateway role); the rank process
                # decides when the whole job has drained, then asks for the counts
                for i in range(nsteps):
                    await publish(i)
                client.send_control({"event": "published", "w": widx})
                cmd = await asyncio.to_thread(client.control.get)
                counts = {k: worker.counts[k] - c0[k] for k in c0}
                counts.update(sink_stored=writer.ok - w0[1], writer_no_merchant=writer.skipped - w0[2],
                              writer_fail=writer.fail - w0[3])
                if profiling:
                    prof.disable()
                    prof_msgs += worker.stage.processed - base
                client.send_control({"event": "done", "w": widx, "s": time.perf_counter() - t0, "counts": counts})
                continue
            pub_task = asyncio.create_task(publish(0)) if nsteps else None
            done_msgs = 0
            for i in range(nsteps):
                if pub_task is not None:
                    await pub_task
                # ingestion of step i+1 overlaps the parsing of step i
                pub_task = asyncio.create_task(publish(i + 1)) if i + 1 < nsteps else None
                done_msgs += len(prepared[i])
                while worker.stage.processed < base + done_msgs:
                    await asyncio.sleep(0.0005)
            if pub_task is not None:
                await pub_task
            # the step ends when the writer has consumed every parsed message too
            parsed = worker.counts["parsed"] - c0["parsed"]
            while writer.stage.processed - w0[0] < parsed:
                await asyncio.sleep(0.0005)
            counts = {k: worker.counts[k] - c0[k] for k in c0}
            counts.update(sink_stored=writer.ok - w0[1], writer_no_merchant=writer.skipped - w0[2],
                          writer_fail=writer.fail - w0[3])
            if profiling:
                prof.disable()
                prof_msgs += worker.stage.processed - base
            client.send_control({"event": "done", "w": widx, "s": time.perf_counter() - t0, "counts": counts})
    if prof is not None:
        import json as _json

        os.makedirs(cfg["profile_dir"], exist_ok=True)
        stem = os.path.join(cfg["profile_dir"], f"parser-r{rank}-w{widx}")
        if hasattr(prof, "dump_stats"):
            prof.dump_stats(stem + ".pstats")
            with open(stem + ".json", "w") as fh:
                _json.dump({"msgs": prof_msgs}, fh)
        else:
            prof.dump(stem + ".samples.json", msgs=prof_msgs)
    await writer.stop()
    await worker.stop()


# ------------------------------------------------------------- HTTP ingest loaders
def spawn_loaders(n: int, rank: int, cfg: Dict[str, Any]) -> Tuple[List[Any], List[Connection]]:
    """Start ``n`` phone-side loader processes (``bench.py --ingest http``): each POSTs
    its share of the prepared SMS to the node's native ``POST /sms/raw`` doors
    (smsgate-busd ``--http-listen``, the reference's api_gateway contract,
    /root/reference/services/api_gateway/main.py:106-134) instead of the parser
    processes publishing to the bus themselves."""
    ctx = mp.get_context("spawn")
    procs, conns = [], []
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    try:
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
        for w in range(n):
            a, b = ctx.Pipe(duplex=True)
            p = ctx.Process(target=loader_main, args=(b, rank, w, cfg), name=f"loader-r{rank}-l{w}", daemon=True)
            p.start()
            b.close()
            procs.append(p)
            conns.append(a)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return procs, conns


def _http_request(path: str, body: bytes) -> bytes:
    return (f"POST {path} HTTP/1.1\r\nHost: smsgate\r\nContent-Type: application/json\r\n"
            f"Content-Length: {len(body)}\r\n\r\n").encode() + body


async def _post_all(doors: Sequence[str], reqs: Sequence[Tuple[bytes, int]], conns: int) -> Dict[str, int]:
    """Send every request over ``conns`` keep-alive HTTP/1.1 connections (spread over
    the doors), one in flight per connection; count 202s and messages accepted."""
    stats = {"requests": 0, "accepted": 0, "rejected": 0}
    nxt = [0]

    async def one(k: int) -> None:
        host, port = doors[k % len(doors)].rsplit(":", 1)
        r, w = await asyncio.open_connection(host, int(port))
        try:
            while nxt[0] < len(reqs):
                req, n = reqs[nxt[0]]
                nxt[0] += 1
                w.write(req)
                await w.drain()
                head = await r.readuntil(b"\r\n\r\n")
                status = int(head.split(b" ", 2)[1])
                clen = 0
                for line in head.split(b"\r\n"):
                    if line[:15].lower() == b"content-length:":
                        clen = int(line[15:])
                if clen:
                    await r.readexactly(clen)
                stats["requests"] += 1
                if status == 202:
                    stats["accepted"] += n
                else:
                    stats["rejected"] += n
        finally:
            w.close()

    await asyncio.gather(*(one(k) for k in range(max(1, conns))))
    return stats


def loader_main(conn: Connection, rank: int, widx: int, cfg: Dict[str, Any]) -> None:
    """A loader process: ``prepare`` builds the HTTP requests (untimed, like the bus
    mode's prepared payloads); ``go`` POSTs them, reports ``published``; ``report``
    answers ``done`` (loaders route nothing: counts stay with the parsers)."""
    import json as _json

    from ..serving import protocol as P

    doors = list(cfg["http_doors"])
    batch = int(cfg.get("http_batch", 1))
    path = "/sms/raw/batch" if batch > 1 else "/sms/raw"
    reqs: List[Tuple[bytes, int]] = []
    stats: Dict[str, int] = {}

    def send(obj: Any) -> None:
        conn.send_bytes(P.pack_control(obj))

    send({"event": "ready", "w": widx})
    while True:
        buf = conn.recv_bytes()
        cmd = P.unpack_control(buf) if P.kind(buf) == b"C" else None
        if cmd is None or cmd.get("cmd") == "quit":
            break
        if cmd["cmd"] == "prepare":
            reqs = []
            for seed in cmd["seeds"]:
                ps = [p.model_dump() for p in _payload_bytes(int(cmd["n"]), seed, cfg.get("vocab", "heldout"),
                                                              cfg.get("traffic", "mixed"))]
                if batch > 1:
                    reqs += [(_http_request(path, _json.dumps(ps[i:i + batch]).encode()), len(ps[i:i + batch]))
                             for i in range(0, len(ps), batch)]
                else:
                    reqs += [(_http_request(path, _json.dumps(p).encode()), 1) for p in ps]
            send({"event": "prepared", "w": widx})
        elif cmd["cmd"] == "go":
            t0 = time.perf_counter()
            stats = asyncio.run(_post_all(doors, reqs, int(cfg.get("http_conns", 8))))
            stats["s"] = time.perf_counter() - t0
            send({"event": "published", "w": widx, "http": stats})
        elif cmd["cmd"] == "report":
            send({"event": "done", "w": widx, "s": stats.get("s", 0.0), "counts": {}, "http": stats})


class Coordinator:
    """Rank-side driver: serves the engine while steering the parser processes.

    With a shared broker (``bus_dsn``) the end of a phase is global: every raw
    message of every rank published (a never-consumed counter durable on
    ``sms.raw`` sees them all) and both the parser and the writer groups drained
    (no pending, nothing un-acked); each rank polls that between engine steps."""

    COUNTER = "bench_raw_counter"
    DRAIN_CHECK_S = 0.02

    def __init__(self, engine, conns: Sequence[Connection], bus_dsn: Optional[str] = None,
                 node_ranks: int = 1) -> None:
        """``node_ranks``: the ranks whose parser processes publish into THIS node's
        broker (LOCAL_WORLD_SIZE: each node starts its own brokers, so a multi-node
        job's drain target counts only the node's own ranks)."""
        from ..serving.remote import EngineServer

        self.events: Dict[str, Dict[int, Any]] = {}
        self.last_http: Dict[str, int] = {}  # HTTP loaders' totals of the last phase
        self.server = EngineServer(engine, conns, on_control=self._on_control)
        self.n = len(conns)
        self.node_ranks = node_ranks
        self.bus = None
        if bus_dsn:
            from ..bus.base import SUBJECT_RAW
            from ..bus.sync_client import SyncBusClient

            self.bus = SyncBusClient(bus_dsn)
            self.bus.ensure_stream()
            self.bus.subscribe(SUBJECT_RAW, self.COUNTER)

    def _drained(self, target_raw: int) -> bool:
        """Every raw message of the phase published and both groups idle.  Each check is
        blocking round trips from the GPU feeder's loop, so they go to the partitions of
        the durable's own subject only, and the groups are asked only once the counter
        has seen every message."""
        from ..bus.base import SUBJECT_PARSED, SUBJECT_RAW

        ci = self.bus.consumer_info
        if ci("SMS", self.COUNTER, subject=SUBJECT_RAW)["num_pending"] < target_raw:
            return False
        for durable, subject in (("parser_worker", SUBJECT_RAW), ("pb_writer", SUBJECT_PARSED)):
            try:
                i = ci("SMS", durable, subject=subject)
            except Exception:  # not created yet
                return False
            if i["num_pending"] or i["num_ack_pending"]:
                return False
        return True

    def _on_control(self, idx: int, obj: Any) -> None:
        self.events.setdefault(obj.get("event", "?"), {})[idx] = obj
        if "http" in obj and obj.get("event") == "done":
            for k, v in obj["http"].items():
                if k != "s":
                    self.last_http[k] = self.last_http.get(k, 0) + int(v)

    def wait_all(self, event: str, timeout: float = 1800.0) -> Dict[int, Any]:
        t_end = time.time() + timeout
        self.server.serve_until(lambda: len(self.events.get(event, {})) >= self.n or time.time() > t_end)
        got = self.events.pop(event, {})
        if len(got) < self.n:
            raise TimeoutError(f"only {len(got)}/{self.n} parser workers reported {event!r}")
        return got

    def broadcast(self, obj: Any) -> None:
        for i in range(self.n):
            self.server.send_control(i, obj)

    def run_phase(self, seeds_per_worker: Sequence[Sequence[int]], n_per_step,
                  sync=None, profile: bool = False) -> Tuple[float, Dict[str, int]]:
        """Prepare (untimed), then time ``go`` → all ``done``. Returns (seconds, routing counts).
        ``n_per_step``: messages per step and connection (an int, or one per connection).
        ``profile``: the parser processes profile this phase (when they were started with
        a profile_dir)."""
        self.last_http = {}
        per = [n_per_step] * self.n if isinstance(n_per_step, int) else list(n_per_step)
        for i in range(self.n):
            self.server.send_control(i, {"cmd": "prepare", "n": per[i], "seeds": list(seeds_per_worker[i])})
        self.wait_all("prepared")
        target = 0
        if self.bus is not None:
            n_raw = sum(len(s) * k for s, k in zip(seeds_per_worker, per)) * self.node_ranks
            target = self.bus.consumer_info("SMS", self.COUNTER)["num_pending"] + n_raw
        if sync is not None:
            sync()
        t0 = time.perf_counter()
        self.broadcast({"cmd": "go", "profile": bool(profile)})
        if self.bus is not None:
            self.wait_all("published")
            last = [0.0]

            def drained() -> bool:
                # a check costs blocking broker round trips in the loop that feeds the
                # GPU: every 20 ms (<= 0.1 % of a 20 s phase added at the end)
                now = time.perf_counter()
                if now - last[0] < self.DRAIN_CHECK_S:
                    return False
                last[0] = now
                return self._drained(target)

            self.server.serve_until(drained)
            if sync is not None:
                sync()
            dt = time.perf_counter() - t0
            self.broadcast({"cmd": "report"})
            done = self.wait_all("done")
        else:
            done = self.wait_all("done")
            if sync is not None:
                sync()
            dt = time.perf_counter() - t0
        counts: Dict[str, int] = {}
        for d in done.values():
            for k, v in d["counts"].items():
                counts[k] = counts.get(k, 0) + v
        return dt, counts

    def shutdown(self, procs: Sequence[Any]) -> None:
        try:
            self.broadcast({"cmd": "quit"})
        except Exception:
            pass
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.terminate()
