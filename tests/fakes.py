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

    def __init__(self, email: str = "a@b.c", password: str = "pw", fail_first: int = 0) -> None:
        self.email, self.password = email, password
        self.cols: Dict[str, List[Dict[str, Any]]] = {}
        self.calls: List[str] = []
        self.fail_first = fail_first
        self._n = 0

    def transport(self) -> httpx.MockTransport:
        return httpx.MockTransport(self.handle)

    def handle(self, req: httpx.Request) -> httpx.Response:
        path = req.url.path
        self.calls.append(f"{req.method} {path}")
        if self.fail_first > 0 and "/records" in path:
            self.fail_first -= 1
            return httpx.Response(503, json={"message": "unavailable"})
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
            fm = re.match(r"msg_id='(.*)'", flt)
            if fm:
                sel = [r for r in items if r.get("msg_id") == fm.group(1)]
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
            self._n += 1
            rec["id"] = f"r{self._n}"
            items.append(rec)
            return httpx.Response(200, json=rec)
        if req.method == "PATCH":
            for r in items:
                if r["id"] == rid:
                    r.update(json.loads(req.content))
                    return httpx.Response(200, json=r)
            return httpx.Response(404)
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
