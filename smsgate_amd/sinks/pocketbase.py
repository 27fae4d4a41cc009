"""PocketBase REST client and sink (libs/pocketbase.py of the reference).

* :meth:`PocketBaseClient.upsert` — GET ``/api/collections/{c}/records?filter=msg_id='…'``
  then PATCH the first hit or POST a new record; retried 5× with exponential
  backoff 2–30 s (pocketbase.py:69-100).
* :meth:`PocketBaseClient.get_records_since` — paginated GET (``perPage=500``,
  ``sort=datetime``, ``filter=datetime > '…'``) until ``page >= totalPages``
  (pocketbase.py:102-128).
* :func:`parsed_to_pb_record` — the record shape written to ``sms_data``
  (pocketbase.py:296-309).

Fixes: the client actually authenticates when credentials are configured
(superuser endpoint of PocketBase ≥ 0.23, then the legacy admin endpoint — D5;
the reference stored ``_token`` and never used it), filter values are quoted
safely, and there is one client class (async) plus a thin sync facade instead
of two copy-pasted clients and a duplicated ``get_pb_client``.

Throughput: the reference's upsert costs two HTTP round trips per record (GET by
filter, then POST/PATCH).  :meth:`PocketBaseClient.batch_upsert` writes up to 50
records in TWO requests (PocketBase ≥ 0.23, batch API enabled): one list query
for the chunk's msg_ids (``msg_id='a' || msg_id='b' …``), then one ``POST
/api/batch`` in which a msg_id already stored is a ``PATCH`` of the record that
holds it (whatever its id: the reference's writer lets PocketBase pick ids) and a
new one is a ``PUT`` on the id derived from its msg_id (:func:`record_id`).  The
per-record path creates records with that same derived id, so the two paths never
write one msg_id twice -- also on the reference schema, whose msg_id index is not
unique (pb_schema.json:149).  The sink falls back to the per-record path for a
chunk the server refuses (batch API disabled -> per-record from then on).
``scripts/sink_bench.py`` measures both paths.
"""
from __future__ import annotations

import asyncio
import logging
from typing import Any, Dict, List, Mapping, Optional, Sequence

import httpx

from ..models.domain import ParsedSMS
from ..runtime.retry import RetryError, retry
from .base import Sink

__all__ = ["PocketBaseClient", "SyncPocketBaseClient", "PocketBaseSink", "parsed_to_pb_record", "COLLECTION_DEBIT",
           "record_id", "PB_BATCH_MAX"]

PB_BATCH_MAX = 50  # PocketBase's default batch.maxRequests

log = logging.getLogger(__name__)

COLLECTION_DEBIT = "sms_data"
COLLECTION_CREDIT = "transactions"


def _q(v: str) -> str:
    return "'" + v.replace("\\", "\\\\").replace("'", "\\'") + "'"


def record_id(msg_id: str) -> str:
    """Deterministic 15-character PocketBase record id ([a-z0-9]) for a msg_id: the
    same SMS always lands on the same record, so an upsert needs no lookup."""
    import hashlib

    return hashlib.sha256(msg_id.encode("utf-8")).hexdigest()[:15]


def parsed_to_pb_record(p: ParsedSMS) -> Dict[str, Any]:
    return {
        "msg_id": p.msg_id,
        "original_body": p.raw_body,
        "sender": p.sender,
        "datetime": p.date.isoformat(),
        "card": p.card,
        "amount": str(p.amount),
        "currency": p.currency,
        "balance": str(p.balance) if p.balance is not None else None,
        "merchant": p.merchant,
        "address": p.address,
        "city": p.city,
        "txn_type": p.txn_type.value,
    }


class PocketBaseClient:
    """Async client for the PocketBase endpoints the pipeline uses."""

    def __init__(self, *, base_url: str, email: str = "", password: str = "", timeout: float = 10.0,
                 transport: Optional[httpx.AsyncBaseTransport] = None,
                 retry_attempts: int = 5, retry_min: float = 2.0, retry_max: float = 30.0) -> None:
        self._base_url = base_url.rstrip("/")
        self._email = email
        self._password = password
        self._client = httpx.AsyncClient(base_url=self._base_url, timeout=timeout, transport=transport)
        self._token: Optional[str] = None
        self._auth_lock = asyncio.Lock()
        self._retry = dict(attempts=retry_attempts, wait_min=retry_min, wait_max=retry_max)
        self.upsert = retry(**self._retry)(self._upsert_once)  # type: ignore[method-assign]

    async def _ensure_auth(self) -> None:
        if self._token is not None or not (self._email and self._password):
            return
        async with self._auth_lock:
            if self._token is not None:
                return
            body = {"identity": self._email, "password": self._password}
            for path in ("/api/collections/_superusers/auth-with-password", "/api/admins/auth-with-password"):
                try:
                    r = await self._client.post(path, json=body)
                except httpx.HTTPError as exc:
                    log.warning("PocketBase auth via %s failed: %s", path, exc)
                    continue
                if r.status_code == 200 and "token" in r.json():
                    self._token = r.json()["token"]
                    self._client.headers["Authorization"] = self._token
                    return
            log.warning("PocketBase auth failed; continuing unauthenticated (public collection rules)")
            self._token = ""

    async def _upsert_once(self, collection: str, record: Mapping[str, Any], *, msg_id: str) -> str:
        await self._ensure_auth()
        params = {"filter": f"msg_id={_q(msg_id)}", "page": 1, "perPage": 1}
        r = await self._client.get(f"/api/collections/{collection}/records", params=params)
        r.raise_for_status()
        items = r.json().get("items", [])
        if items:
            rec_id = items[0]["id"]
            r = await self._client.patch(f"/api/collections/{collection}/records/{rec_id}", json=dict(record))
            r.raise_for_status()
            return "patched"
        # created under the msg_id-derived id, the id the batch path PUTs: both paths
        # address one record per msg_id
        r = await self._client.post(f"/api/collections/{collection}/records",
                                    json={"id": record_id(msg_id), **dict(record)})
        r.raise_for_status()
        return "created"

    async def existing_ids(self, collection: str, msg_ids: Sequence[str]) -> Dict[str, str]:
        """msg_id -> id of a record already holding it (one list request per call)."""
        uniq = list(dict.fromkeys(msg_ids))
        if not uniq:
            return {}
        params = {"filter": " || ".join(f"msg_id={_q(m)}" for m in uniq), "page": 1,
                  "perPage": max(len(uniq) * 2, 30), "fields": "id,msg_id"}
        r = await self._client.get(f"/api/collections/{collection}/records", params=params)
        r.raise_for_status()
        out: Dict[str, str] = {}
        for it in r.json().get("items", []):
            out.setdefault(str(it.get("msg_id")), str(it["id"]))
        return out

    async def batch_upsert(self, collection: str, records: Sequence[Mapping[str, Any]]) -> Optional[bool]:
        """Upsert ``records`` (each with its ``msg_id``) in one ``POST /api/batch``.
        Returns True when stored, False when the server refused this batch (the
        caller retries it per record), None when the server has no batch API."""
        await self._ensure_auth()
        try:
            have = await self.existing_ids(collection, [str(r["msg_id"]) for r in records])
        except httpx.HTTPError as exc:
            log.warning("PocketBase msg_id lookup failed: %s", exc)
            return False
        reqs = []
        for rec in records:
            m = str(rec["msg_id"])
            if m in have:
                reqs.append({"method": "PATCH", "url": f"/api/collections/{collection}/records/{have[m]}",
                             "body": dict(rec)})
            else:
                reqs.append({"method": "PUT", "url": f"/api/collections/{collection}/records",
                             "body": {"id": record_id(m), **dict(rec)}})
                have[m] = record_id(m)  # a repeated msg_id in the same chunk updates that record
        try:
            r = await self._client.post("/api/batch", json={"requests": reqs})
        except httpx.HTTPError as exc:
            log.warning("PocketBase batch request failed: %s", exc)
            return False
        if r.status_code in (403, 404, 405):  # batch API disabled / absent (PocketBase < 0.23)
            return None
        return r.status_code == 200

    async def get_records_since(self, collection: str, since_pb_str: str, per_page: int = 500) -> List[Dict[str, Any]]:
        await self._ensure_auth()
        items: List[Dict[str, Any]] = []
        page = 1
        while True:
            params = {"page": page, "perPage": per_page, "sort": "datetime", "filter": f"datetime > {_q(since_pb_str)}"}
            r = await self._client.get(f"/api/collections/{collection}/records", params=params)
            r.raise_for_status()
            data = r.json()
            batch = data.get("items", [])
            if not batch:
                break
            items.extend(batch)
            if data.get("page", page) >= data.get("totalPages", page):
                break
            page += 1
        return items

    async def close(self) -> None:
        await self._client.aclose()

    async def __aenter__(self) -> "PocketBaseClient":
        return self

    async def __aexit__(self, *exc: Any) -> None:
        await self.close()


class SyncPocketBaseClient:
    """Blocking facade (the reference's sync ``PocketBaseClient``)."""

    def __init__(self, **kw: Any) -> None:
        self._kw = kw

    def _run(self, name: str, *a: Any, **kw: Any) -> Any:
        async def go():
            async with PocketBaseClient(**self._kw) as c:
                return await getattr(c, name)(*a, **kw)

        return asyncio.run(go())

    def upsert(self, collection: str, record: Mapping[str, Any], *, msg_id: str) -> str:
        return self._run("upsert", collection, record, msg_id=msg_id)

    def get_records_since(self, collection: str, since_pb_str: str) -> List[Dict[str, Any]]:
        return self._run("get_records_since", collection, since_pb_str)


class PocketBaseSink(Sink):
    name = "pocketbase"

    def __init__(self, client: PocketBaseClient, collection: str = COLLECTION_DEBIT, concurrency: int = 8,
                 batch: int = PB_BATCH_MAX) -> None:
        self.client = client
        self.collection = collection
        self._sem = asyncio.Semaphore(concurrency)
        self.batch = max(1, min(batch, PB_BATCH_MAX))
        self.batch_supported: Optional[bool] = None if self.batch > 1 else False  # None = not probed yet
        self.batched = 0  # records written through /api/batch
        self.per_record = 0  # records written with GET + POST/PATCH

    async def _one(self, p: ParsedSMS) -> None:
        async with self._sem:
            try:
                await self.client.upsert(self.collection, parsed_to_pb_record(p), msg_id=p.msg_id)
            except RetryError:
                log.error("PocketBase upsert gave up for %s", p.msg_id)
                raise

    async def _chunk(self, chunk: Sequence[ParsedSMS]) -> None:
        if self.batch_supported is not False and len(chunk) > 1:
            async with self._sem:
                ok = await self.client.batch_upsert(self.collection, [parsed_to_pb_record(p) for p in chunk])
            if ok is None:
                log.info("PocketBase has no batch API: writing one record at a time")
                self.batch_supported = False
            elif ok:
                self.batch_supported = True
                self.batched += len(chunk)
                return
        res = await asyncio.gather(*(self._one(p) for p in chunk), return_exceptions=True)
        self.per_record += len(chunk)
        errs = [r for r in res if isinstance(r, BaseException)]
        if errs:
            raise errs[0]

    async def upsert_many(self, records: Sequence[ParsedSMS]) -> None:
        chunks = [records[i:i + self.batch] for i in range(0, len(records), self.batch)]
        errs: List[BaseException] = []
        if self.batch_supported is None and len(chunks) > 1:
            # probe the batch API with the first chunk before fanning out the rest
            try:
                await self._chunk(chunks[0])
            except BaseException as exc:  # noqa: BLE001
                errs.append(exc)
            chunks = chunks[1:]
        res = await asyncio.gather(*(self._chunk(c) for c in chunks), return_exceptions=True)
        errs += [r for r in res if isinstance(r, BaseException)]
        if errs:
            raise errs[0]

    async def close(self) -> None:
        await self.client.close()
