"""Offline batch tools of the pre-bus era, re-implemented on the framework.

The reference ships four root scripts — two of them broken
(``save_to_pocketbase.py`` SyntaxError, ``loader.py`` NameError, D14).  Same
capabilities, working, on the in-repo sqlite KV instead of ``diskcache``:

* :func:`import_xml_to_cache`   — read_xml.py: SMS backup XML → cache keyed by ``date``;
* :func:`process_cache`         — process_cached.py: rule-based parsing of every cached
  SMS into a debit and a credit cache, OTP skipped, per-record ``status``;
* :func:`sync_to_pocketbase`    — save_to_pocketbase.py: push both result caches to the
  ``sms_data`` / ``transactions`` collections with msg-id dedup, mark ``synced``;
* :func:`fetch_hookdeck_events` — loader.py: page through the Hookdeck events API
  (``/2024-03-01/events``, limit 100, cursor pagination), cache events by id and
  parse their message text.

Unlike the legacy regexes, parsing reuses :func:`extract_rule_based`, which
gets city/address right and handles the multi-line format.
"""
from __future__ import annotations

import hashlib
import json
import xml.etree.ElementTree as ET
from pathlib import Path
from typing import Any, Dict, List, Optional

import httpx

from ..parse.backends.regex import extract_rule_based
from ..parse.cache import SqliteKV
from ..parse.text import normalize_body

__all__ = ["import_xml_to_cache", "process_cache", "sync_to_pocketbase", "fetch_hookdeck_events"]


def import_xml_to_cache(xml_path: str | Path, cache: SqliteKV) -> int:
    root = ET.parse(xml_path).getroot()
    n = 0
    items = []
    for el in root.findall("sms"):
        attrs = dict(el.attrib)
        key = attrs.get("date")
        if not key:
            continue
        items.append((key, attrs))
        n += 1
    cache.put_many(items)
    return n


def _otp(body: str) -> bool:
    up = body.upper()
    return "OTP" in up or "PASS=" in up or "CODE:" in up


def process_cache(source: SqliteKV, purchases: SqliteKV, credits: SqliteKV) -> Dict[str, int]:
    stats = {"processed_debit": 0, "processed_credit": 0, "failed": 0, "skipped": 0}
    updates: List = []
    for key, rec in source.items():
        if rec.get("status") in ("processed", "skipped_otp"):
            stats["skipped"] += 1
            continue
        body = (rec.get("body") or "").strip()
        if _otp(body):
            rec["status"] = "skipped_otp"
            stats["skipped"] += 1
        else:
            ans = extract_rule_based(normalize_body(body))
            if ans is None:
                rec["status"] = "failed"
                stats["failed"] += 1
            else:
                out = dict(ans, source_key=key, body=body, msg_id=hashlib.md5(body.encode()).hexdigest())
                if ans["txn_type"] == "credit":
                    credits.put(key, out)
                    stats["processed_credit"] += 1
                else:
                    purchases.put(key, out)
                    stats["processed_debit"] += 1
                rec["status"] = "processed"
        updates.append((key, rec))
    source.put_many(updates)
    return stats


async def sync_to_pocketbase(purchases: SqliteKV, credits: SqliteKV, pb) -> Dict[str, int]:
    """``pb`` is a :class:`~smsgate_amd.sinks.pocketbase.PocketBaseClient`."""
    stats = {"sms_data": 0, "transactions": 0, "skipped": 0}
    for cache, collection in ((purchases, "sms_data"), (credits, "transactions")):
        marks = []
        for key, rec in cache.items():
            if rec.get("status") == "synced":
                stats["skipped"] += 1
                continue
            record = {k: rec.get(k) for k in ("msg_id", "merchant", "city", "address", "card", "amount", "currency",
                                                "balance", "txn_type")}
            record["datetime"] = rec.get("date")
            record["original_body"] = rec.get("body")
            await pb.upsert(collection, record, msg_id=rec["msg_id"])
            rec["status"] = "synced"
            marks.append((key, rec))
            stats[collection] += 1
        cache.put_many(marks)
    return stats


async def fetch_hookdeck_events(api_key: str, webhook_id: Optional[str], cache: SqliteKV,
                                transport: Optional[httpx.AsyncBaseTransport] = None,
                                base_url: str = "https://api.hookdeck.com") -> Dict[str, int]:
    stats = {"events": 0, "parsed": 0}
    params: Dict[str, Any] = {"limit": 100}
    if webhook_id:
        params["webhook_id"] = webhook_id
    async with httpx.AsyncClient(base_url=base_url, transport=transport, timeout=30,
                                 headers={"Authorization": f"Bearer {api_key}"}) as c:
        while True:
            r = await c.get("/2024-03-01/events", params=params)
            r.raise_for_status()
            data = r.json()
            items = []
            for ev in data.get("models", []):
                body = ev.get("data", {}).get("body") if isinstance(ev.get("data"), dict) else None
                text = body.get("message") if isinstance(body, dict) else (body if isinstance(body, str) else None)
                ev["parsed"] = extract_rule_based(normalize_body(text)) if text else None
                stats["parsed"] += ev["parsed"] is not None
                items.append((str(ev.get("id")), ev))
            cache.put_many(items)
            stats["events"] += len(items)
            nxt = (data.get("pagination") or {}).get("next")
            if not nxt or not items:
                break
            params["next"] = nxt
    return stats


def dump_cache(cache: SqliteKV) -> str:
    return json.dumps(dict(cache.items()), ensure_ascii=False, indent=2)
