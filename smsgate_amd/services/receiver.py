"""Webhook capture server (receiver.py parity).

The reference runs a stdlib ``HTTPServer`` on a random localhost port behind an
ngrok tunnel: ``POST`` stores the raw body in a disk cache under a fresh
uuid4 key and answers **201** ``{"status": "success", "message": "Webhook
received and stored.", "key": <uuid>}``; ``GET`` lists the stored keys
(``{"message": "Listing stored webhook keys.", "count": n, "keys": [...]}``)
(receiver.py:30-88).  Here the store is the in-repo sqlite KV (``diskcache``
is absent) and the app is FastAPI; ``GET /{key}`` additionally returns one
stored body.  Tunnelling is left to the deployment (no ngrok SDK on the image).
"""
from __future__ import annotations

import base64
import sqlite3
import threading
import uuid
from pathlib import Path
from typing import List, Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse

__all__ = ["BlobStore", "create_receiver_app"]


class BlobStore:
    """sqlite-backed key → bytes store (the role of ``diskcache.Cache('.hookdeck_cache')``)."""

    def __init__(self, path: str | Path) -> None:
        self._db = sqlite3.connect(str(path), check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("CREATE TABLE IF NOT EXISTS blobs (k TEXT PRIMARY KEY, v BLOB NOT NULL, ts REAL)")
        self._lock = threading.Lock()

    def set(self, key: str, value: bytes) -> None:
        import time

        with self._lock:
            self._db.execute("INSERT OR REPLACE INTO blobs (k, v, ts) VALUES (?, ?, ?)", (key, value, time.time()))

    def get(self, key: str) -> Optional[bytes]:
        with self._lock:
            r = self._db.execute("SELECT v FROM blobs WHERE k = ?", (key,)).fetchone()
        return None if r is None else bytes(r[0])

    def keys(self) -> List[str]:
        with self._lock:
            return [r[0] for r in self._db.execute("SELECT k FROM blobs ORDER BY ts")]

    def close(self) -> None:
        self._db.close()


def create_receiver_app(store: BlobStore) -> FastAPI:
    app = FastAPI(title="Webhook receiver")

    @app.post("/{path:path}")
    async def post_any(path: str, request: Request):
        body = await request.body()
        key = str(uuid.uuid4())
        store.set(key, body)
        return JSONResponse({"status": "success", "message": "Webhook received and stored.", "key": key},
                            status_code=201)

    @app.get("/")
    async def list_keys():
        keys = store.keys()
        return {"message": "Listing stored webhook keys.", "count": len(keys), "keys": keys}

    @app.get("/{key}")
    async def get_one(key: str):
        v = store.get(key)
        if v is None:
            return JSONResponse({"error": "not found"}, status_code=404)
        try:
            return {"key": key, "body": v.decode("utf-8")}
        except UnicodeDecodeError:
            return {"key": key, "body_b64": base64.b64encode(v).decode()}

    return app
