"""In-process fakes of the external HTTP services (PocketBase, Telegram, Gemini, Hookdeck)
served through ``httpx.MockTransport`` — no network on the image."""
from __future__ import annotations

import json
import re
from typing import Any, Dict, List
from urllib.parse import parse_qs

import httpx


class FakePocketBase:
    """Enough of the PocketBase REST API: superuser auth, list with ``msg_id=`` /
    ``datetime >`` filters + sort + pagination, create, patch."""

    def __init__(self, email: str = "a@b.c", password: str = "pw", fail_first: int = 0,
                 batch_enabled: bool = False, unique_msg_id: bool = True) -> None:
        self.email, self.password = email, password
        self.cols: Dict[str, List[Dict[str, Any]]] = {}
        self.calls: List[str] = []
        self.fail_first = fail_first
        self.batch_enabled = batch_enabled  # PocketBase >= 0.23 batch API (off by default there too)
        self.unique_msg_id = unique_msg_id  # deploy/pb_schema.json: unique msg_id index
        self._n = 0
        self._idx: Dict[str, Dict[str, Any]] = {}

    def _batch(self, req: httpx.Request) -> httpx.Response:
        """POST /api/batch: all-or-nothing; PUT = upsert by the body's id."""
        if not self.batch_enabled:
            return httpx.Response(403, json={"message": "Batch requests are not allowed."})
        reqs = json.loads(req.content)["requests"]
        plan = []  # validate everything first (all-or-nothing), then apply
        seen_msg = {}
        for r in reqs:
            um = re.match(r"/api/collections/([^/]+)/records(?:/([^/]+))?$", r["url"])
            col = um.group(1)
            items = self.cols.setdefault(col, [])
            idx = self._index(col)
            body = dict(r["body"])
            if r["method"] == "PATCH":
                if um.group(2) not in idx["id"]:
                    return httpx.Response(404, json={"message": "not found"})
                body["id"] = um.group(2)
            hit = idx["id"].get(body["id"])
            if hit is None and self.unique_msg_id:
                owner = idx["msg"].get(body.get("msg_id"), seen_msg.get((col, body.get("msg_id"))))
                if owner is not None and owner != body["id"]:
                    return httpx.Response(400, json={"message": "msg_id: value must be unique"})
            seen_msg[(col, body.get("msg_id"))] = body["id"]
            plan.append((col, items, idx, hit, body))
        for col, items, idx, hit, body in plan:
            if hit is None:
                hit = idx["id"].get(body["id"])
            if hit is None:
                items.append(body)
                idx["id"][body["id"]] = body
            else:
                hit.update(body)
            idx["msg"][body.get("msg_id")] = body["id"]
        return httpx.Response(200, json=[{"status": 200, "body": b} for *_, b in plan])

    def _index(self, col):
        """id -> record and msg_id -> id of a collection (rebuilt if the list was replaced)."""
        items = self.cols.setdefault(col, [])
        idx = self._idx.get(col)
        if idx is None or idx["list"] is not items or idx["n"] != len(items):
            idx = {"list": items, "n": len(items), "id": {r["id"]: r for r in items},
                   "msg": {r.get("msg_id"): r["id"] for r in items}}
            self._idx[col] = idx
        return idx

    def transport(self) -> httpx.MockTransport:
        return httpx.MockTransport(self.handle)

    def handle(self, req: httpx.Request) -> httpx.Response:
        path = req.url.path
        self.calls.append(f"{req.method} {path}")
        if self.fail_first > 0 and "/records" in path:
            self.fail_first -= 1
            return httpx.Response(503, json={"message": "unavailable"})
        if path == "/api/batch":
            return self._batch(req)
        if path.endswith("auth-with-password"):
            body = json.loads(req.content)
            if body == {"identity": self.email, "password": self.password}:
                return httpx.Response(200, json={"token": "T0K"})
            return httpx.Response(400, json={"message": "bad"})
        m = re.match(r"/api/collections/([^/]+)/records(?:/([^/]+))?$", path)
        if not m:
            return httpx.Response(404)
        col, rid = m.group(1), m.group(2)
        items = self.cols.setdefault(col, [])
        if req.method == "GET":
            q = {k: v[0] for k, v in parse_qs(req.url.query.decode()).items()}
            flt = q.get("filter", "")
            sel = items
            if flt.startswith("msg_id="):
                wanted = set(re.findall(r"msg_id='((?:[^'\\]|\\.)*)'", flt))
                # every record holding one of the msg_ids (duplicates included: the
                # reference schema's msg_id index is not unique)
                sel = [r for r in items if r.get("msg_id") in wanted]
            fm = re.match(r"datetime > '(.*)'", flt)
            if fm:
                sel = [r for r in items if str(r.get("datetime", "")) > fm.group(1)]
            if q.get("sort") == "datetime":
                sel = sorted(sel, key=lambda r: str(r.get("datetime", "")))
            page, per = int(q.get("page", 1)), int(q.get("perPage", 30))
            total_pages = max(1, -(-len(sel) // per))
            return httpx.Response(200, json={"page": page, "perPage": per, "totalPages": total_pages,
                                             "totalItems": len(sel), "items": sel[(page - 1) * per: page * per]})
        if req.method == "POST":
            rec = json.loads(req.content)
            idx = self._index(col)
            if "id" not in rec:  # PocketBase picks a random id when the client sends none
                self._n += 1
                rec["id"] = f"r{self._n}"
            elif rec["id"] in idx["id"]:
                return httpx.Response(400, json={"message": "id: value must be unique"})
            if self.unique_msg_id and rec.get("msg_id") in idx["msg"]:
                return httpx.Response(400, json={"message": "msg_id: value must be unique"})
            items.append(rec)
            idx["id"][rec["id"]] = rec
            idx["msg"][rec.get("msg_id")] = rec["id"]
            idx["n"] = len(items)
            return httpx.Response(200, json=rec)
        if req.method == "PATCH":
            r = self._index(col)["id"].get(rid)
            if r is None:
                return httpx.Response(404)
            r.update(json.loads(req.content))
            return httpx.Response(200, json=r)
        return httpx.Response(405)


class FakeTelegram:
    def __init__(self, updates: List[Dict[str, Any]] | None = None) -> None:
        self.sent: List[Dict[str, Any]] = []
        self.updates = list(updates or [])

    def transport(self) -> httpx.MockTransport:
        return httpx.MockTransport(self.handle)

    def handle(self, req: httpx.Request) -> httpx.Response:
        method = req.url.path.rsplit("/", 1)[-1]
        if method == "getUpdates":
            ups, self.updates = self.updates, []
            return httpx.Response(200, json={"ok": True, "result": ups})
        ctype = req.headers.get("content-type", "")
        info: Dict[str, Any] = {"method": method, "bytes": len(req.content)}
        if "multipart" in ctype:
            txt = req.content.decode("utf-8", "ignore")
            info["chat_id"] = int(re.search(r'name="chat_id"\r\n\r\n(-?\d+)', txt).group(1))
            cap = re.search(r'name="caption"\r\n\r\n(.*?)\r\n--', txt, re.S)
            info["caption"] = cap.group(1) if cap else ""
        else:
            form = {k: v[0] for k, v in parse_qs(req.content.decode()).items()}
            info["chat_id"] = int(form["chat_id"])
            info["text"] = form.get("text", "")
        self.sent.append(info)
        return httpx.Response(200, json={"ok": True, "result": {}})
