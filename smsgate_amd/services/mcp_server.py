"""MCP (Model Context Protocol) server exposing the ``sms_data`` table as tools.

Parity with services/mcp_server/server.py (FastMCP "SQLAlchemy DB Connector",
SSE transport on 0.0.0.0:9122): the same six tools with the same arguments and
result shapes —

* ``get_record_by_id(record_id)`` → row dict | ``{"error": …}``
* ``find_sms_records(sender, card, txn_type, min_amount, max_amount, start_date, end_date)``
  → list of rows (AND of the given filters; ISO dates)
* ``update_record_by_id(record_id, updates)`` → message string
* ``delete_record_by_id(record_id)`` → message string
* ``create_parsed_sms(parsed_sms_data)`` → message string (idempotent upsert by msg_id)
* ``get_current_datetime()`` → local ISO-8601 time

The ``mcp`` SDK is not installed on the image, so the protocol is implemented
directly (JSON-RPC 2.0: ``initialize``, ``tools/list``, ``tools/call``,
``ping``) on FastAPI with both transports: legacy SSE (``GET /sse`` +
``POST /messages?session_id=…``, what FastMCP's ``transport="sse"`` serves)
and streamable HTTP (``POST /mcp``).
"""
from __future__ import annotations

import asyncio
import datetime as _dt
import json
import uuid
from decimal import Decimal
from typing import Any, Dict, Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, StreamingResponse

from ..db.schema import sms_data
from ..models.domain import ParsedSMS

__all__ = ["McpTools", "create_mcp_app", "TOOL_SPECS", "PROTOCOL_VERSION"]

PROTOCOL_VERSION = "2024-11-05"
SERVER_NAME = "SQLAlchemy DB Connector"

INSTRUCTIONS = (
    "This server provides tools to interact with 'sms_data' records directly in the database. "
    "create_parsed_sms, get_record_by_id, find_sms_records, update_record_by_id, delete_record_by_id, "
    "get_current_datetime."
)

_num = {"type": ["number", "null"]}
_str = {"type": ["string", "null"]}
TOOL_SPECS: Dict[str, Dict[str, Any]] = {
    "get_record_by_id": {"description": "Retrieve one sms_data record by primary key id.",
                         "inputSchema": {"type": "object", "properties": {"record_id": {"type": "integer"}},
                                         "required": ["record_id"]}},
    "find_sms_records": {"description": "Find sms_data records (AND of filters; ISO dates).",
                         "inputSchema": {"type": "object", "properties": {
                             "sender": _str, "card": _str, "txn_type": _str, "min_amount": _num,
                             "max_amount": _num, "start_date": _str, "end_date": _str}}},
    "update_record_by_id": {"description": "Update fields of an sms_data record by id.",
                            "inputSchema": {"type": "object", "properties": {
                                "record_id": {"type": "integer"}, "updates": {"type": "object"}},
                                "required": ["record_id", "updates"]}},
    "delete_record_by_id": {"description": "Delete an sms_data record by id.",
                            "inputSchema": {"type": "object", "properties": {"record_id": {"type": "integer"}},
                                            "required": ["record_id"]}},
    "create_parsed_sms": {"description": "Create or update a parsed SMS record (msg_id is the unique key).",
                          "inputSchema": {"type": "object", "properties": {"parsed_sms_data": {"type": "object"}},
                                          "required": ["parsed_sms_data"]}},
    "get_current_datetime": {"description": "Current local time in ISO-8601.",
                             "inputSchema": {"type": "object", "properties": {}}},
}


def _jsonable(v: Any) -> Any:
    if isinstance(v, Decimal):
        return str(v)
    if isinstance(v, (_dt.datetime, _dt.date)):
        return v.isoformat()
    return v


def _row(r: Dict[str, Any]) -> Dict[str, Any]:
    return {k: _jsonable(v) for k, v in r.items()}


class McpTools:
    """The six tools over a :class:`~smsgate_amd.sinks.sql.SqlSink`."""

    def __init__(self, sink) -> None:
        self.sink = sink

    async def get_record_by_id(self, record_id: int) -> Dict[str, Any]:
        try:
            r = await asyncio.to_thread(self.sink.get_by_id, int(record_id))
            return _row(r) if r else {"error": f"Record with ID '{record_id}' not found in 'sms_data' collection."}
        except Exception as e:  # noqa: BLE001
            return {"error": f"Failed to retrieve record: {e}"}

    async def find_sms_records(self, sender: Optional[str] = None, card: Optional[str] = None,
                               txn_type: Optional[str] = None, min_amount: Optional[float] = None,
                               max_amount: Optional[float] = None, start_date: Optional[str] = None,
                               end_date: Optional[str] = None) -> Any:
        c = sms_data.c
        conds = []
        if sender:
            conds.append(c.sender == sender)
        if card:
            conds.append(c.card == card)
        if txn_type:
            conds.append(c.txn_type == txn_type)
        if min_amount is not None:
            conds.append(c.amount >= Decimal(str(min_amount)))
        if max_amount is not None:
            conds.append(c.amount <= Decimal(str(max_amount)))
        for val, op, name in ((start_date, ">=", "start_date"), (end_date, "<=", "end_date")):
            if val:
                try:
                    d = _dt.datetime.fromisoformat(val)
                except ValueError:
                    return {"error": f"Invalid {name} format. Use ISO 8601 (e.g., '2024-01-01T00:00:00')."}
                conds.append(c.datetime >= d if op == ">=" else c.datetime <= d)
        try:
            rows = await asyncio.to_thread(self.sink.find, conds)
            return [_row(r) for r in rows]
        except Exception as e:  # noqa: BLE001
            return {"error": f"Failed to find records: {e}"}

    async def update_record_by_id(self, record_id: int, updates: Dict[str, Any]) -> str:
        unknown = sorted(set(updates) - set(sms_data.c.keys()) | ({"id"} & set(updates)))
        if unknown:
            return f"Failed to update record: unknown or read-only column(s) {unknown}"
        try:
            upd = dict(updates)
            for k in ("amount", "balance"):
                if upd.get(k) is not None:
                    upd[k] = Decimal(str(upd[k]))
            if isinstance(upd.get("datetime"), str):
                upd["datetime"] = _dt.datetime.fromisoformat(upd["datetime"])
            n = await asyncio.to_thread(self.sink.update_by_id, int(record_id), upd)
            if n == 0:
                return f"Record with ID '{record_id}' not found in 'sms_data' collection. No update performed."
            return f"Record '{record_id}' in 'sms_data' collection updated successfully."
        except Exception as e:  # noqa: BLE001
            return f"Failed to update record: {e}"

    async def delete_record_by_id(self, record_id: int) -> str:
        try:
            n = await asyncio.to_thread(self.sink.delete_by_id, int(record_id))
            if n == 0:
                return f"Record with ID '{record_id}' not found in 'sms_data' collection. No deletion performed."
            return f"Record '{record_id}' deleted successfully from 'sms_data' collection."
        except Exception as e:  # noqa: BLE001
            return f"Failed to delete record: {e}"

    async def create_parsed_sms(self, parsed_sms_data: Dict[str, Any]) -> str:
        try:
            p = ParsedSMS.model_validate(parsed_sms_data)
            await self.sink.upsert_many([p])
            return f"Parsed SMS record with msg_id '{p.msg_id}' successfully created/updated."
        except Exception as e:  # noqa: BLE001
            return f"Failed to create/update parsed SMS record: {e}"

    async def get_current_datetime(self) -> str:
        return _dt.datetime.now().astimezone().isoformat()

    async def call(self, name: str, args: Dict[str, Any]) -> Any:
        if name not in TOOL_SPECS:
            raise KeyError(name)
        return await getattr(self, name)(**(args or {}))


async def handle_rpc(tools: McpTools, msg: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """One JSON-RPC 2.0 message → response (None for notifications)."""
    mid = msg.get("id")
    method = msg.get("method")
    params = msg.get("params") or {}

    def ok(result):
        return {"jsonrpc": "2.0", "id": mid, "result": result}

    def err(code, text):
        return {"jsonrpc": "2.0", "id": mid, "error": {"code": code, "message": text}}

    if mid is None:  # notification (e.g. notifications/initialized)
        return None
    if method == "initialize":
        return ok({"protocolVersion": PROTOCOL_VERSION, "capabilities": {"tools": {"listChanged": False}},
                   "serverInfo": {"name": SERVER_NAME, "version": "0.1.0"}, "instructions": INSTRUCTIONS})
    if method == "ping":
        return ok({})
    if method == "tools/list":
        return ok({"tools": [{"name": n, **spec} for n, spec in TOOL_SPECS.items()]})
    if method == "tools/call":
        name = params.get("name")
        try:
            res = await tools.call(name, params.get("arguments") or {})
        except KeyError:
            return err(-32602, f"unknown tool {name!r}")
        except TypeError as e:
            return err(-32602, f"bad arguments: {e}")
        text = res if isinstance(res, str) else json.dumps(res, ensure_ascii=False, default=str)
        is_err = isinstance(res, dict) and "error" in res
        return ok({"content": [{"type": "text", "text": text}], "isError": is_err,
                   "structuredContent": res if not isinstance(res, str) else {"result": res}})
    return err(-32601, f"method not found: {method}")


def create_mcp_app(tools: McpTools) -> FastAPI:
    app = FastAPI(title=SERVER_NAME)
    sessions: Dict[str, asyncio.Queue] = {}

    @app.post("/mcp")
    async def mcp_http(request: Request):
        body = await request.json()
        if isinstance(body, list):
            out = [r for r in [await handle_rpc(tools, m) for m in body] if r is not None]
            return JSONResponse(out) if out else JSONResponse(None, status_code=202)
        r = await handle_rpc(tools, body)
        return JSONResponse(r) if r is not None else JSONResponse(None, status_code=202)

    @app.get("/sse")
    async def sse(request: Request):
        sid = uuid.uuid4().hex
        q: asyncio.Queue = asyncio.Queue()
        sessions[sid] = q

        async def events():
            yield f"event: endpoint\ndata: /messages/?session_id={sid}\n\n"
            try:
                while True:
                    if await request.is_disconnected():
                        break
                    try:
                        msg = await asyncio.wait_for(q.get(), 15.0)
                        yield f"event: message\ndata: {json.dumps(msg, ensure_ascii=False, default=str)}\n\n"
                    except asyncio.TimeoutError:
                        yield ": ping\n\n"
            finally:
                sessions.pop(sid, None)

        return StreamingResponse(events(), media_type="text/event-stream")

    @app.post("/messages/")
    async def messages(session_id: str, request: Request):
        q = sessions.get(session_id)
        if q is None:
            return JSONResponse({"error": "unknown session"}, status_code=404)
        r = await handle_rpc(tools, await request.json())
        if r is not None:
            await q.put(r)
        return JSONResponse({"status": "accepted"}, status_code=202)

    return app
