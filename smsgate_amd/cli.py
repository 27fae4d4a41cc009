"""``python -m smsgate_amd <service> [options]`` — one entry point per service.

The reference starts each service from its own Dockerfile CMD / launch.json
entry: ``api_gateway``, ``parser_worker --name --group``,
``dlq_worker --group --reparse``, ``pb_writer``, ``xml_watcher``,
``dashboard``, ``mcp_server``, plus the root scripts and ``make`` alembic
targets.  Subcommands here:

==================  ==========================================================
gateway             FastAPI ingestion (uvicorn) — API_HOST/API_PORT
parser              parser worker (``--group``, ``--backend``, ``--engine``)
writer              sms.parsed → PocketBase (if PB_URL set) + SQL (DATABASE_URL)
dlq                 DLQ inspector (``--reparse``)
xml-watcher         BACKUP_DIR poller
notifier            PocketBase → chart → Telegram
mcp-server          MCP tools over SSE / streamable HTTP (port 9122)
receiver            webhook capture server
bus-server          durable broker (``--listen``, ``--data``, ``--native`` = C++ smsgate-busd)
engine-server       GPU extraction engine for parser processes (``--listen``)
pipeline            gateway + parser + writer in one process (memory bus)
db                  migrations: upgrade|downgrade|current|history|stamp
legacy              import-xml | process-cache | sync-pb | hookdeck
config              print the effective settings
==================  ==========================================================
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import socket
import sys
from typing import List, Optional

__all__ = ["main"]

log = logging.getLogger("smsgate")


def _stop_event() -> asyncio.Event:
    ev = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, ev.set)
        except (NotImplementedError, RuntimeError):
            pass
    return ev


def _pipeline(settings, backend_name: Optional[str] = None, engine: Optional[str] = None):
    from .parse.backends import create_backend
    from .parse.cache import open_cache
    from .parse.pipeline import ParsePipeline
    from .parse.text import set_keyword_match

    set_keyword_match(settings.parser_keyword_match)
    name = backend_name or settings.parser_backend
    if engine:
        from multiprocessing.connection import Client

        from .parse.backends.local_llm import RemoteLLMBackend
        from .serving.remote import RemoteEngineClient

        path = engine.replace("unix://", "")
        # the connector lets the client reconnect after an engine-server restart
        client = RemoteEngineClient(connector=lambda: Client(path, family="AF_UNIX"))
        backend = RemoteLLMBackend(client, max_batch=settings.parser_batch_size)
    else:
        backend = create_backend(name)
    return ParsePipeline(backend, open_cache(settings.parser_cache_path))


def _sinks(settings):
    from .sinks.sql import SqlSink

    sinks = []
    if settings.pb_url and os.getenv("PB_URL"):
        from .sinks.pocketbase import PocketBaseClient, PocketBaseSink

        sinks.append(PocketBaseSink(PocketBaseClient(base_url=settings.pb_url, email=settings.pb_email,
                                                     password=settings.pb_password)))
    sinks.append(SqlSink(_sql_url(settings)))
    return sinks


def _sql_url(settings, override: Optional[str] = None) -> str:
    """DATABASE_URL → Postgres (when POSTGRES_HOST is configured) → local sqlite file."""
    url = override or settings.database_url_override
    if not url and os.getenv("POSTGRES_HOST"):
        url = settings.database_url
    return url or "sqlite:///smsgate.sqlite"


async def _run_parser(a, settings) -> None:
    from .bus import connect
    from .obs.errors import init_sentry
    from .obs.metrics import start_metrics_server
    from .services.parser import ParserWorker

    start_metrics_server(settings.parser_metrics_port)
    init_sentry(release="parser_worker@2.0.0")
    bus = await connect(settings.nats_dsn)
    w = ParserWorker(bus, _pipeline(settings, a.backend, a.engine), group=a.group,
                     concurrency=a.concurrency or settings.parser_concurrency, batch=settings.parser_batch_size)
    log.info("parser worker %s in group %s (backend %s)", a.name, a.group, w.pipeline.backend.name)
    await w.run(_stop_event())
    await bus.drain()


async def _run_writer(a, settings) -> None:
    from .bus import connect
    from .obs.errors import init_sentry
    from .obs.metrics import start_metrics_server
    from .services.writer import WriterService

    init_sentry(release="pb_writer@2.0.0")
    start_metrics_server(int(os.getenv("PBWRITER_METRICS_PORT", settings.pbwriter_metrics_port)))
    bus = await connect(settings.nats_dsn)
    await WriterService(bus, _sinks(settings)).run(_stop_event())


async def _run_dlq(a, settings) -> None:
    from .bus import connect
    from .services.dlq import DlqWorker

    bus = await connect(settings.nats_dsn)
    # --reparse re-runs the REAL parser (dlq_worker.py:59-78): with --engine the GPU
    # engine-server the parsers use (an outage naks the batch, it never drops it)
    w = DlqWorker(bus, _pipeline(settings, a.backend, a.engine) if a.reparse else None, group=a.group,
                  reparse=a.reparse)
    await w.start()
    await _stop_event().wait()
    await w.stop()


async def _run_xml(a, settings) -> None:
    from .bus import connect
    from .services.xml_watcher import XmlWatcher

    bus = await connect(settings.nats_dsn)
    await XmlWatcher(bus, settings.backup_dir, settings.xml_scan_interval_s).run(_stop_event())


async def _run_notifier(a, settings) -> None:
    from pathlib import Path

    from .services.notifier import Notifier, NotifierState, TelegramClient
    from .sinks.pocketbase import PocketBaseClient

    pb = PocketBaseClient(base_url=settings.pb_url, email=settings.pb_email, password=settings.pb_password)
    n = Notifier(pb, TelegramClient(settings.tg_bot_token), settings.allowed_chat_ids,
                 NotifierState(Path(a.state)), Path(a.out_dir), settings.check_interval_seconds)
    await n.run(_stop_event())


async def _run_bus_server(a, settings) -> None:
    from .bus.server import serve

    native = getattr(a, "native", False)
    await serve(a.listen, a.data, _stop_event(), max_age=settings.stream_max_age_s,
                nats_listen=a.nats_listen, native=native, http_listen=a.http_listen)


async def _run_pipeline(a, settings) -> None:
    import uvicorn

    from .bus import MemoryBus
    from .services.gateway import create_app
    from .services.parser import ParserWorker
    from .services.writer import WriterService

    bus = MemoryBus()

    async def get_bus():
        return bus

    parser = ParserWorker(bus, _pipeline(settings, a.backend))
    writer = WriterService(bus, _sinks(settings))
    await parser.start()
    await writer.start()
    cfg = uvicorn.Config(create_app(get_bus, log_dir=settings.log_dir), host=settings.api_host or "0.0.0.0",
                         port=int(settings.api_port or 9001), log_level="info")
    await uvicorn.Server(cfg).serve()
    await parser.stop()
    await writer.stop()


def _engine_server(a) -> None:
    import threading

    from .parse.backends.local_llm import build_engine
    from .serving.remote import EngineServer

    from .config import get_settings
    from .parse.backends.local_llm import MissingCheckpoint, resolve_checkpoint

    st = get_settings()
    model = a.model or st.llm_model
    try:  # before touching the GPU: no trained weights -> exit non-zero, never serve random ones silently
        ckpt = resolve_checkpoint(model, a.checkpoint or st.llm_checkpoint, a.random_init)
    except MissingCheckpoint as exc:
        log.error("engine-server: %s", exc)
        raise SystemExit(2) from exc
    if ckpt is None:
        log.warning("engine-server: serving RANDOM-INIT weights (--random-init): answers are meaningless")
    from .serving.profiles import profile_kwargs

    kw = profile_kwargs(a.profile, max_slots=a.max_slots)
    eng = build_engine(model, ckpt, a.device, random_init=a.random_init, **kw)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    path = a.listen.replace("unix://", "")
    if os.path.exists(path):
        os.unlink(path)
    log.info("engine server on %s (%s, %s, profile %s, %d slots)", a.listen, model, ckpt or "random-init",
             a.profile, eng.cfg.max_slots)
    from .obs.metrics import EngineMetricsExporter, start_metrics_server

    start_metrics_server(env_var="ENGINE_METRICS_PORT", default=9104)
    exporter = EngineMetricsExporter(eng).start()
    from .serving import freeze_gc_for_launch_loop

    freeze_gc_for_launch_loop()
    try:
        EngineServer(eng).serve_listener(path, stop)
    finally:
        exporter.stop()


def train_config(a, world: int = 1):
    """The :class:`TrainConfig` of ``train-extractor`` arguments: the flagship recipe
    (models/train.py FLAGSHIP_RECIPE -- what bench.py trains and measures) with the
    given overrides; ``--batch`` is the global batch, split over ``world`` ranks."""
    from .models.train import recipe

    return recipe(a.model, a.steps, a.batch, world=world, lr=a.lr, n_examples=a.examples, seed=a.seed,
                  ckpt_dir=a.ckpt_dir, ckpt_every=a.ckpt_every, resume=a.resume, bucket_mb=a.bucket_mb,
                  answer_format=a.answer_format, families=None if a.families == "legacy" else a.families,
                  negatives=a.negatives)


def _train(a, settings) -> None:
    """``train-extractor``; under ``torchrun --nproc-per-node N`` one rank per GPU
    (RCCL data parallel, :mod:`smsgate_amd.parallel.ddp`)."""
    import torch
    import torch.distributed as dist

    from .models.train import train_extractor

    world = int(os.environ.get("WORLD_SIZE", "1"))
    device = settings.llm_device
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            device = f"cuda:{local}"
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(device))
        else:
            device = "cpu"
            dist.init_process_group("gloo")
    cfg = train_config(a, world)
    w = train_extractor(cfg, device=device)
    if not dist.is_initialized() or dist.get_rank() == 0:
        w.save(a.out)
        print(f"saved {a.out}")
    if dist.is_initialized():
        dist.destroy_process_group()


def _db(a, settings) -> None:
    from .db import migrations
    from .sinks.sql import make_engine

    eng = make_engine(_sql_url(settings, a.url))
    if a.action == "upgrade":
        print(migrations.upgrade(eng, a.target or "head"))
    elif a.action == "downgrade":
        print(migrations.downgrade(eng, a.target or "-1"))
    elif a.action == "current":
        print(migrations.current(eng))
    elif a.action == "history":
        print("\n".join(migrations.history()))
    elif a.action == "stamp":
        migrations.stamp(eng, a.target or migrations.HEAD)


async def _legacy(a, settings) -> None:
    from .parse.cache import SqliteKV
    from .services import legacy

    if a.action == "import-xml":
        print(legacy.import_xml_to_cache(a.xml, SqliteKV(a.cache)))
    elif a.action == "process-cache":
        print(legacy.process_cache(SqliteKV(a.cache), SqliteKV(a.purchases), SqliteKV(a.credits)))
    elif a.action == "sync-pb":
        from .sinks.pocketbase import PocketBaseClient

        async with PocketBaseClient(base_url=settings.pb_url, email=settings.pb_email,
                                    password=settings.pb_password) as pb:
            print(await legacy.sync_to_pocketbase(SqliteKV(a.purchases), SqliteKV(a.credits), pb))
    elif a.action == "hookdeck":
        print(await legacy.fetch_hookdeck_events(os.environ["HOOKDECK_API_KEY"], os.getenv("HOOKDECK_WEBHOOK_ID"),
                                                 SqliteKV(a.cache)))


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m smsgate_amd", description="smsgate_amd services")
    p.add_argument("-v", "--verbose", action="store_true")
    sp = p.add_subparsers(dest="cmd", required=True)
    gp = sp.add_parser("gateway")
    gp.add_argument("--workers", type=int, default=0,
                    help="HTTP worker processes on the port (default GATEWAY_WORKERS or 1)")
    pp = sp.add_parser("parser")
    pp.add_argument("--name", default=f"{socket.gethostname()}-{os.getpid()}")
    pp.add_argument("--group", default="parser_worker")
    pp.add_argument("--backend", default=None)
    pp.add_argument("--engine", default=None, help="unix:///path of an engine-server (GPU)")
    pp.add_argument("--concurrency", type=int, default=0)
    sp.add_parser("writer")
    dp = sp.add_parser("dlq")
    dp.add_argument("--name", default=f"{socket.gethostname()}-{os.getpid()}")
    dp.add_argument("--group", default="parser_worker_dlq")
    dp.add_argument("--reparse", action="store_true")
    dp.add_argument("--backend", default=None, help="parser backend for --reparse (default PARSER_BACKEND)")
    dp.add_argument("--engine", default=None, help="unix:///path of an engine-server (GPU) for --reparse")
    sp.add_parser("xml-watcher")
    np_ = sp.add_parser("notifier")
    np_.add_argument("--state", default="last_state.json")
    np_.add_argument("--out-dir", default=".")
    mp_ = sp.add_parser("mcp-server")
    mp_.add_argument("--url", default=None)
    rp = sp.add_parser("receiver")
    rp.add_argument("--cache", default=".hookdeck_cache.sqlite")
    rp.add_argument("--port", type=int, default=0)
    bp = sp.add_parser("bus-server")
    bp.add_argument("--listen", default="tcp://0.0.0.0:4223", help="msgpack protocol (tcp:// or unix://)")
    bp.add_argument("--nats-listen", default="tcp://0.0.0.0:4222", help="NATS wire protocol ('' = off)")
    bp.add_argument("--data", default="./.bus-data")
    bp.add_argument("--native", action="store_true",
                    help="run the C++ broker (smsgate-busd: msgpack + NATS protocols, same journal format)")
    bp.add_argument("--http-listen", default="",
                    help="with --native: native HTTP ingestion (POST /sms/raw, /sms/raw/batch, /health, /metrics)")
    ep = sp.add_parser("engine-server")
    ep.add_argument("--listen", default="unix:///tmp/smsgate-engine0.sock")
    ep.add_argument("--model", default=None, help="default: LLM_MODEL (smollm-135m)")
    ep.add_argument("--checkpoint", default=None, help="safetensors weights (default: LLM_CHECKPOINT)")
    ep.add_argument("--random-init", action="store_true",
                    help="serve random weights (throughput tests only; every SMS ends in the DLQ)")
    ep.add_argument("--device", default="cuda:0")
    ep.add_argument("--profile", default="throughput", choices=["throughput", "latency"],
                    help="engine configuration (serving/profiles.py): the one bench.py measures by default")
    ep.add_argument("--max-slots", type=int, default=None, help="default: the profile's")
    pl = sp.add_parser("pipeline")
    pl.add_argument("--backend", default=None)
    db = sp.add_parser("db")
    db.add_argument("action", choices=["upgrade", "downgrade", "current", "history", "stamp"])
    db.add_argument("target", nargs="?")
    db.add_argument("--url", default=None)
    lg = sp.add_parser("legacy")
    lg.add_argument("action", choices=["import-xml", "process-cache", "sync-pb", "hookdeck"])
    lg.add_argument("--xml")
    lg.add_argument("--cache", default="sms_cache.sqlite")
    lg.add_argument("--purchases", default="parsed_sms_cache.sqlite")
    lg.add_argument("--credits", default="credit_sms_cache.sqlite")
    from .models.train import FLAGSHIP_RECIPE as R

    tr = sp.add_parser("train-extractor", help="train the local extractor LM on synthetic SMS (GPU); the defaults "
                       "are the flagship recipe bench.py trains and measures (models/train.py FLAGSHIP_RECIPE)")
    tr.add_argument("--model", default=R.model)
    tr.add_argument("--steps", type=int, default=R.steps)
    tr.add_argument("--batch", type=int, default=R.batch, help="GLOBAL batch (split over torchrun ranks)")
    tr.add_argument("--lr", type=float, default=R.lr)
    tr.add_argument("--examples", type=int, default=0, help="training examples (0 = steps x batch, all fresh)")
    tr.add_argument("--seed", type=int, default=R.seed)
    tr.add_argument("--out", required=True, help="safetensors path (LLM_CHECKPOINT for the local_llm backend)")
    tr.add_argument("--ckpt-dir", default=None, help="training checkpoints (weights + optimizer + step)")
    tr.add_argument("--ckpt-every", type=int, default=0)
    tr.add_argument("--resume", action="store_true", help="continue from the newest checkpoint in --ckpt-dir")
    tr.add_argument("--bucket-mb", type=float, default=64.0, help="DP gradient all-reduce bucket size")
    tr.add_argument("--answer-format", default=R.answer_format, choices=["copy", "span", "qa", "qa17"],
                    help="qa: the whole answer from one forward (serving/qa.py); span: two pointer decode steps "
                         "per copied field; copy: the body's tokens (the checkpoint records it; the engine follows)")
    tr.add_argument("--negatives", type=float, default=R.negatives,
                    help="share of non-transaction examples (txn_type unknown / otp, null fields)")
    tr.add_argument("--families", default="train", help="train (every training SMS layout) | legacy (the two "
                    "reference formats only)")
    sp.add_parser("config")
    return p


def main(argv: Optional[List[str]] = None) -> int:
    a = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if a.verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    from .config import get_settings

    settings = get_settings()
    if a.cmd == "config":
        print(settings.dump())
    elif a.cmd == "gateway":
        import uvicorn

        from .obs.errors import init_sentry
        from .services.gateway import create_app

        from .services.tunnel import open_tunnel

        init_sentry(release="api_gateway@0.1.0")
        port = int(settings.api_port or 9001)
        tunnel = open_tunnel(settings, port)
        workers = a.workers or int(os.getenv("GATEWAY_WORKERS", "1"))
        try:
            if workers > 1:
                # N processes on one port (SO_REUSEPORT), each with its own bus client;
                # Prometheus counters aggregated across them (services/gateway_runner.py)
                from .services.gateway_runner import serve_workers

                serve_workers(workers, settings.api_host or "0.0.0.0", port)
            else:
                uvicorn.run(create_app(log_dir=settings.log_dir), host=settings.api_host or "0.0.0.0", port=port)
        finally:
            if tunnel is not None:
                tunnel.close()
    elif a.cmd == "parser":
        asyncio.run(_run_parser(a, settings))
    elif a.cmd == "writer":
        asyncio.run(_run_writer(a, settings))
    elif a.cmd == "dlq":
        asyncio.run(_run_dlq(a, settings))
    elif a.cmd == "xml-watcher":
        asyncio.run(_run_xml(a, settings))
    elif a.cmd == "notifier":
        asyncio.run(_run_notifier(a, settings))
    elif a.cmd == "mcp-server":
        import uvicorn

        from .services.mcp_server import McpTools, create_mcp_app
        from .sinks.sql import SqlSink

        sink = SqlSink(_sql_url(settings, a.url))
        uvicorn.run(create_mcp_app(McpTools(sink)), host=settings.mcp_host, port=settings.mcp_port)
    elif a.cmd == "receiver":
        import uvicorn

        from .services.receiver import BlobStore, create_receiver_app

        uvicorn.run(create_receiver_app(BlobStore(a.cache)), host="127.0.0.1", port=a.port or 8088)
    elif a.cmd == "bus-server":
        asyncio.run(_run_bus_server(a, settings))
    elif a.cmd == "engine-server":
        _engine_server(a)
    elif a.cmd == "pipeline":
        asyncio.run(_run_pipeline(a, settings))
    elif a.cmd == "db":
        _db(a, settings)
    elif a.cmd == "legacy":
        asyncio.run(_legacy(a, settings))
    elif a.cmd == "train-extractor":
        _train(a, settings)
    return 0


if __name__ == "__main__":
    sys.exit(main())
