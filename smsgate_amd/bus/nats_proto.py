"""NATS client protocol (text framing) + the JetStream API subset the pipeline uses.

Shared by :mod:`.nats_client` (our services against a real ``nats-server``) and
:mod:`.nats_server` (our durable broker answering NATS clients).  Core protocol:
``INFO``/``CONNECT``/``PUB``/``HPUB``/``SUB``/``UNSUB``/``MSG``/``HMSG``/
``PING``/``PONG``/``+OK``/``-ERR``, CRLF-terminated control lines, sized
payloads; headers are ``NATS/1.0[ <status> <text>]\\r\\n(Key: Value\\r\\n)*\\r\\n``.

JetStream is plain request/reply on ``$JS.API.*`` subjects with JSON bodies
(durations in nanoseconds) and acks published to the delivery's reply subject
``$JS.ACK.<stream>.<consumer>.<delivered>.<stream_seq>.<consumer_seq>.<ts_ns>.<pending>``.
The reference drives exactly this through nats-py (libs/nats_utils.py:50-129,
worker.py:197-224, writer.py:93-100, dlq_worker.py:84-90).
"""
from __future__ import annotations

import asyncio
import json
import os
import secrets
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

CRLF = b"\r\n"
HDR_LINE = b"NATS/1.0"
API = "$JS.API"
ACK_PREFIX = "$JS.ACK."
MAX_PAYLOAD = 8 * 1024 * 1024


def nuid(n: int = 22) -> str:
    alphabet = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
    raw = secrets.token_bytes(n)
    return "".join(alphabet[b % 62] for b in raw)


def new_inbox() -> str:
    return f"_INBOX.{nuid()}"


def encode_headers(headers: Optional[Dict[str, str]], status: Optional[str] = None) -> bytes:
    line = HDR_LINE + (b" " + status.encode() if status else b"")
    out = [line]
    for k, v in (headers or {}).items():
        out.append(f"{k}: {v}".encode())
    return CRLF.join(out) + CRLF + CRLF


def decode_headers(raw: bytes) -> Tuple[Optional[int], str, Dict[str, str]]:
    """-> (status code or None, status text, headers)."""
    lines = raw.split(CRLF)
    first = lines[0].decode(errors="replace")
    status: Optional[int] = None
    text = ""
    rest = first[len("NATS/1.0"):].strip()
    if rest:
        code, _, text = rest.partition(" ")
        if code.isdigit():
            status = int(code)
    hdrs: Dict[str, str] = {}
    for ln in lines[1:]:
        if not ln:
            continue
        k, _, v = ln.decode(errors="replace").partition(":")
        hdrs[k.strip()] = v.strip()
    return status, text, hdrs


@dataclass
class Frame:
    op: str  # MSG | HMSG | PUB | HPUB | SUB | UNSUB | INFO | CONNECT | PING | PONG | +OK | -ERR
    args: List[str]
    payload: bytes = b""
    headers: bytes = b""


async def read_frame(reader: asyncio.StreamReader) -> Frame:
    """One protocol operation (both directions: the sized ops carry their payload)."""
    line = await reader.readuntil(CRLF)
    line = line[:-2]
    if not line:
        return Frame("", [])
    head, _, tail = line.partition(b" ")
    op = head.decode().upper()
    if op in ("INFO", "CONNECT", "-ERR"):
        return Frame(op, [tail.decode(errors="replace")])
    args = tail.decode(errors="replace").split()
    if op in ("MSG", "PUB"):
        size = int(args[-1])
        data = await reader.readexactly(size + 2)
        return Frame(op, args[:-1], data[:-2])
    if op in ("HMSG", "HPUB"):
        hsize, total = int(args[-2]), int(args[-1])
        data = await reader.readexactly(total + 2)
        return Frame(op, args[:-2], data[hsize:total], data[:hsize])
    return Frame(op, args)


def pub_bytes(subject: str, payload: bytes, reply: Optional[str] = None,
              headers: Optional[bytes] = None) -> bytes:
    r = f" {reply}" if reply else ""
    if headers:
        return (f"HPUB {subject}{r} {len(headers)} {len(headers) + len(payload)}\r\n".encode()
                + headers + payload + CRLF)
    return f"PUB {subject}{r} {len(payload)}\r\n".encode() + payload + CRLF


def msg_bytes(subject: str, sid: str, payload: bytes, reply: Optional[str] = None,
              headers: Optional[bytes] = None) -> bytes:
    r = f" {reply}" if reply else ""
    if headers:
        return (f"HMSG {subject} {sid}{r} {len(headers)} {len(headers) + len(payload)}\r\n".encode()
                + headers + payload + CRLF)
    return f"MSG {subject} {sid}{r} {len(payload)}\r\n".encode() + payload + CRLF


# ------------------------------------------------------------------ JetStream JSON
NS = 1_000_000_000


def stream_config_json(cfg) -> Dict[str, Any]:
    return {
        "name": cfg.name,
        "subjects": list(cfg.subjects),
        "retention": "limits",
        "max_consumers": -1,
        "max_msgs": cfg.max_msgs,
        "max_bytes": cfg.max_bytes,
        "max_age": int(cfg.max_age * NS),
        "max_msg_size": -1,
        "storage": cfg.storage,
        "discard": "old",
        "num_replicas": 1,
    }


def stream_config_from_json(d: Dict[str, Any]):
    from .base import StreamConfig

    return StreamConfig(name=d["name"], subjects=list(d.get("subjects") or [d["name"]]),
                        max_age=float(d.get("max_age", 0)) / NS, max_msgs=int(d.get("max_msgs", -1)),
                        max_bytes=int(d.get("max_bytes", -1)), storage=d.get("storage", "file"))


def parse_ack_subject(subject: str) -> Optional[Dict[str, Any]]:
    """``$JS.ACK.<stream>.<consumer>.<delivered>.<sseq>.<cseq>.<ts>.<pending>`` (v1, 9 tokens)
    or the v2 form with ``<domain>.<account hash>`` after ACK (12 tokens, trailing token)."""
    t = subject.split(".")
    if len(t) == 9:
        s, c, dlv, sseq, cseq, ts, pend = t[2:9]
    elif len(t) >= 11:
        s, c, dlv, sseq, cseq, ts, pend = t[4:11]
    else:
        return None
    return {"stream": s, "consumer": c, "delivered": int(dlv), "stream_seq": int(sseq),
            "consumer_seq": int(cseq), "timestamp": int(ts), "pending": int(pend)}


def api_error(code: int, err_code: int, description: str) -> Dict[str, Any]:
    return {"error": {"code": code, "err_code": err_code, "description": description}}


def dumps(obj: Any) -> bytes:
    return json.dumps(obj, separators=(",", ":")).encode()


def server_id() -> str:
    return "NSMSGATE" + os.urandom(8).hex().upper()
