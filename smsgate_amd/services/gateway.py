"""HTTP ingestion gateway (FastAPI) — ``services/api_gateway/main.py`` parity.

Endpoints and exact responses (api_gateway/main.py:106-157):

* ``POST /sms/raw`` — body ``{"device_id", "message", "sender", "timestamp": int,
  "source": str|null}`` (schemas.py:21-25; FastAPI answers 422 on a schema
  mismatch). It is mapped to :class:`RawSMS` with ``msg_id = md5(message)``,
  ``body = message``, ``date = str(timestamp)``; a domain-validation failure
  (empty sender/body, ``source`` not ``device``/``xml`` — including a missing
  ``source``, whose DTO default ``None`` fails, a kept quirk) answers
  **400 {"detail": "Invalid payload"}**; a publish failure **500
  {"detail": "Internal error"}**; success **202 {"result": "queued"}**.
* ``GET /health`` — **200 {"status": "ok"}** when the bus answers a real ping
  (the reference only checked that a cached connection object existed),
  else **503 {"status": "redis_down"}** (the body string is a kept contract).

Additions: ``GET /metrics`` (Prometheus — README.md:37 promised it, D12),
``POST /sms/raw/batch`` (one publish round trip for many SMS) and
``GET /debug/errors`` (recent captured errors).  No per-request stream
check: the stream is ensured once at start-up (D3).

Scale: concurrent ``POST /sms/raw`` requests share broker round trips
(:class:`~smsgate_amd.bus.coalesce.PublishCoalescer`; each request still waits
for its own PubAck before the 202), and ``gateway --workers N`` runs N
processes on one port (uvicorn workers; :func:`default_app` is the per-process
factory; Prometheus counters aggregated across them).
"""
from __future__ import annotations

import logging
import time
from contextlib import asynccontextmanager
from pathlib import Path
from typing import Any, Awaitable, Callable, List, Optional

from fastapi import FastAPI, HTTPException, Request, status
from fastapi.responses import JSONResponse, Response
from pydantic import BaseModel

from ..bus.base import SUBJECT_RAW, Bus
from ..bus.coalesce import PublishCoalescer
from ..models.domain import RawSMS, get_md5_hash, raw_wire
from ..obs import metrics as M
from ..obs.errors import recent_errors, sentry_capture

__all__ = ["RawSMSPayload", "ShortSMSPayload", "RawSMSResponse", "create_app", "payload_to_raw", "default_app"]

log = logging.getLogger("api_gateway")


class RawSMSPayload(BaseModel):
    """What a phone/webhook posts (schemas.py:13-30)."""

    device_id: str
    message: str
    sender: str
    timestamp: int
    source: Optional[str] = None


class ShortSMSPayload(BaseModel):
    """Alternative DTO kept for API-surface parity (schemas.py:32-50; unused there too)."""

    device_id: str
    msg_id: str
    message: str
    sender: str
    timestamp: str
    source: Optional[str] = None


class RawSMSResponse(BaseModel):
    result: str = "queued"


def payload_to_raw(p: RawSMSPayload) -> RawSMS:
    return RawSMS.model_validate(
        {
            "msg_id": get_md5_hash(p.message),
            "sender": p.sender,
            "body": p.message,
            "date": str(p.timestamp),
            "device_id": p.device_id,
            "source": p.source,
        }
    )


BusGetter = Callable[[], Awaitable[Bus]]


def create_app(get_bus: Optional[BusGetter] = None, *, log_dir: Optional[str] = None,
               ensure_stream_on_start: bool = True, coalesce: bool = True) -> FastAPI:
    if get_bus is None:
        from ..bus import connect

        async def get_bus() -> Bus:  # type: ignore[no-redef]
            return await connect()

    if log_dir:
        d = Path(log_dir)
        d.mkdir(parents=True, exist_ok=True)
        fh = logging.FileHandler(d / "api_gateway.log", encoding="utf-8")
        fh.setFormatter(logging.Formatter("%(asctime)s [%(levelname)s] %(name)s: %(message)s"))
        log.addHandler(fh)

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        if ensure_stream_on_start:
            try:
                await (await app.state.get_bus()).ensure_stream()
            except Exception as exc:  # health will report it
                log.warning("bus unavailable at start-up: %s", exc)
        log.info("API gateway started")
        yield
        log.info("API gateway shutting down")

    app = FastAPI(title="SMS API Gateway", version="0.1.0", lifespan=lifespan)
    app.state.get_bus = get_bus
    coalescers: dict = {}

    async def publish_one(bus: Bus, data: bytes) -> None:
        if not coalesce:
            await bus.publish(SUBJECT_RAW, data)
            return
        c = coalescers.get(id(bus))
        if c is None or c.bus is not bus:
            c = coalescers[id(bus)] = PublishCoalescer(bus)
        await c.publish(SUBJECT_RAW, data)

    app.state.coalescers = coalescers

    @app.post("/sms/raw", status_code=status.HTTP_202_ACCEPTED)
    async def post_raw_sms(payload: RawSMSPayload, request: Request) -> JSONResponse:
        try:
            raw = payload_to_raw(payload)
        except Exception as exc:
            log.error("payload validation failed: %s", exc)
            sentry_capture(exc)
            M.GATEWAY_REQUESTS.labels("/sms/raw", "400").inc()
            raise HTTPException(status_code=400, detail="Invalid payload") from exc
        try:
            t0 = time.perf_counter()
            bus = await request.app.state.get_bus()
            await publish_one(bus, raw_wire(raw))
            M.GATEWAY_PUBLISH_TIME.observe(time.perf_counter() - t0)
        except Exception as exc:
            sentry_capture(exc)
            log.exception("failed to publish to the bus")
            M.GATEWAY_REQUESTS.labels("/sms/raw", "500").inc()
            raise HTTPException(status_code=500, detail="Internal error") from exc
        M.GATEWAY_REQUESTS.labels("/sms/raw", "202").inc()
        return JSONResponse(content={"result": "queued"}, status_code=status.HTTP_202_ACCEPTED)

    @app.post("/sms/raw/batch", status_code=status.HTTP_202_ACCEPTED)
    async def post_raw_batch(payloads: List[RawSMSPayload], request: Request) -> JSONResponse:
        try:
            raws = [payload_to_raw(p) for p in payloads]
        except Exception as exc:
            sentry_capture(exc)
            M.GATEWAY_REQUESTS.labels("/sms/raw/batch", "400").inc()
            raise HTTPException(status_code=400, detail="Invalid payload") from exc
        try:
            bus = await request.app.state.get_bus()
            await bus.publish_many([(SUBJECT_RAW, raw_wire(r)) for r in raws])
        except Exception as exc:
            sentry_capture(exc)
            M.GATEWAY_REQUESTS.labels("/sms/raw/batch", "500").inc()
            raise HTTPException(status_code=500, detail="Internal error") from exc
        M.GATEWAY_REQUESTS.labels("/sms/raw/batch", "202").inc()
        return JSONResponse(content={"result": "queued", "count": len(raws)}, status_code=202)

    @app.get("/health", status_code=status.HTTP_200_OK, response_model=None)
    async def health(request: Request) -> Any:
        try:
            bus = await request.app.state.get_bus()
            ok = await bus.ping()
            if not ok:
                raise ConnectionError("bus ping failed")
            return {"status": "ok"}
        except Exception as exc:
            log.error("health check failed: %s", exc)
            sentry_capture(exc)
            return JSONResponse(status_code=status.HTTP_503_SERVICE_UNAVAILABLE, content={"status": "redis_down"})

    @app.get("/metrics")
    async def metrics() -> Response:
        return Response(M.render_latest(), media_type="text/plain; version=0.0.4")

    @app.get("/debug/errors")
    async def debug_errors(n: int = 50) -> Any:
        return recent_errors(n)

    return app


def default_app() -> FastAPI:
    """Per-process app factory of ``gateway --workers N`` (uvicorn ``factory=True``):
    every worker process connects its own bus client from the settings."""
    from ..config import get_settings

    return create_app(log_dir=get_settings().log_dir)
